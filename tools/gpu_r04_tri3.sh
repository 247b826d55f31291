#!/bin/bash
# round 4: branch-free bitmap probe in k_tri_heavy -- parity, then s22 / s24 / s26 benches + s26 trace
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tri_variants.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" tests/test_gpu_api.py > $O/tests.txt 2>&1
echo tests done
for s in 22 24 26; do
  timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 3 --warmup 1 --no-cpu-baseline > $O/s$s.json 2> $O/s$s.err
  echo "s$s done"
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" > $O/tests_s26.txt 2>&1
echo s26 test done
