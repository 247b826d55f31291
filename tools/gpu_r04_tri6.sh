#!/bin/bash
# round 4: k_tri_light prefetch (GS_TH_LPREF_Q / _S variants) at s24 / s26
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t6
mkdir -p $O
for v in lp11 lp00 lp21; do
  lib=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so
  GELLY_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" -k "20 or 22" > $O/tests_$v.txt 2>&1
  for s in 26; do
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 3 --warmup 1 \
      --no-cpu-baseline > $O/${v}_s$s.json 2> $O/${v}_s$s.err
    echo "$v s$s done"
  done
done
