#!/bin/bash
# Runs bench.py once per tuning build under gelly-streaming_amd/variants/*, one JSON line each.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in gelly-streaming_amd/variants/*/; do
  name=$(basename "$v")
  echo "== $name" >> gpurun_out/tune.log
  GELLY_HIP_LIB="$PWD/$v/libgellyhip.so" timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline \
    > "gpurun_out/tune_$name.json" 2>> gpurun_out/tune.log || { echo "FAILED $name rc=$?" >> gpurun_out/tune.log; exit 1; }
done
