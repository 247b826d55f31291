#!/bin/bash
# round 4: 2-byte list tails for the heavy count (GS_TH_NARROW) -- parity, then s24 / s26 A/B
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tri_variants.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" tests/test_gpu_api.py > $O/tests.txt 2>&1
echo tests done
tb() { local name=$1 s=$2; shift 2; env "$@" timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/$name.json 2> $O/$name.err; echo "$name done"; }
tb n1_s24 24 GS_TH_NARROW=1
tb n0_s24 24 GS_TH_NARROW=0
tb n1_s26 26 GS_TH_NARROW=1
tb n0_s26 26 GS_TH_NARROW=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" > $O/tests_s26.txt 2>&1
echo s26 test done
bash tools/gpu_r04_c2ab.sh
echo all done
