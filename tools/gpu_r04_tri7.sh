#!/bin/bash
# round 4: the simplified light path -- every triangle test (variants, C4 shapes, s26, API, dist), then s24 / s26
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t7
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_tri_variants.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" \
  tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_stream.py > $O/tests.txt 2>&1
echo tests done
for s in 24 26; do
  timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 3 --warmup 1 --no-cpu-baseline > $O/s$s.json 2> $O/s$s.err
  echo "s$s done"
done
