#!/bin/bash
# round 4: sampled degree classes by default for windows >= 2^26 edges -- every triangle test (incl. the
# C4 shapes s20-s24 and the s26 window vs the oracle), then s24 / s26 bench lines default vs
# GS_TRI_DEG_SAMPLE=1 (exact degrees), same box
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04degs2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_tri_degree_sample.py \
  tests/test_gpu_tri_variants.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_threads.py \
  tests/test_gpu_stream.py "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" > $O/tests.txt 2>&1
echo tests done
b() { local name=$1 k=$2; shift 2; GS_TRI_DEG_SAMPLE=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload triangles "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b s24_def_1 4 --scale 24
b s24_k1_1 1 --scale 24
b s24_def_2 4 --scale 24
b s24_k1_2 1 --scale 24
b s26_def 4 --scale 26 --steps 3 --warmup 1
b s26_k1 1 --scale 26 --steps 3 --warmup 1
