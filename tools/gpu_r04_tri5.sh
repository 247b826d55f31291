#!/bin/bash
# round 4: light vertices queued by k_tri_lclass (GS_TH_LCLASS) -- parity, then A/B at s22 / s24 / s26
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tri_variants.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" tests/test_gpu_api.py tests/test_gpu_dist.py > $O/tests.txt 2>&1
echo tests done
for s in 24 26; do
  for l in 1 0; do
    GS_TH_LCLASS=$l timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 3 --warmup 1 --no-cpu-baseline \
      > $O/l${l}_s$s.json 2> $O/l${l}_s$s.err
    echo "l$l s$s done"
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" > $O/tests_s26.txt 2>&1
echo s26 test done
bash tools/gpu_r04_tri6.sh
echo tri6 done
