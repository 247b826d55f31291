#!/bin/bash
# round 4 A/B: triangle degree classes from the window's first n/k edges (GS_TRI_DEG_SAMPLE=k; any id
# order gives the exact count) -- the C4-shape parity tests with k = 4, then s24 / s26 bench lines
# alternating k = 1 / 4 / 8, same box
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04degs}
mkdir -p $O
GS_TRI_DEG_SAMPLE=4 timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" > $O/tests_k4.txt 2>&1
echo tests done
b() { local name=$1 k=$2; shift 2; GS_TRI_DEG_SAMPLE=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload triangles "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
for i in 1 2; do
  b s24_k1_$i 1 --scale 24
  b s24_k4_$i 4 --scale 24
  b s24_k8_$i 8 --scale 24
done
b s26_k1 1 --scale 26 --steps 3 --warmup 1
b s26_k4 4 --scale 26 --steps 3 --warmup 1
b s26_k8 8 --scale 26 --steps 3 --warmup 1
