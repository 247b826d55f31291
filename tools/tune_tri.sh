#!/bin/bash
# triangle tuning builds (variants/*): triangle parity tests + s22 bench line each, and the in-tree build
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --workload triangles --scale 24 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ttri_default.json 2>> gpurun_out/ttri.log || exit 1
for v in gelly-streaming_amd/variants/*/; do
  name=$(basename "$v")
  echo "== $name" >> gpurun_out/ttri.log
  GELLY_HIP_LIB="$PWD/$v/libgellyhip.so" timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_api.py -k "triangle" -m gpu >> gpurun_out/ttri.log 2>&1 || { echo "TESTS FAILED $name" >> gpurun_out/ttri.log; exit 1; }
  GELLY_HIP_LIB="$PWD/$v/libgellyhip.so" timeout -k 10 200 python bench.py --workload triangles --scale 24 --steps 2 --warmup 1 --no-cpu-baseline \
    > "gpurun_out/ttri_$name.json" 2>> gpurun_out/ttri.log || { echo "FAILED $name rc=$?" >> gpurun_out/ttri.log; exit 1; }
done
