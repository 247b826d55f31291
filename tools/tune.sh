#!/bin/bash
# Runs bench.py (with --check) once per tuning build under gelly-streaming_amd/variants/*, one JSON line
# each, plus the in-tree build; optional: the bucket tests against every variant (TUNE_TESTS=1).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --check --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/tune_default.json 2>> gpurun_out/tune.log || exit 1
for v in gelly-streaming_amd/variants/*/; do
  name=$(basename "$v")
  echo "== $name" >> gpurun_out/tune.log
  if [ -n "$TUNE_TESTS" ] && [ "${name#abl}" = "$name" ]; then
    GELLY_HIP_LIB="$PWD/$v/libgellyhip.so" timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_bucket.py -m gpu >> gpurun_out/tune.log 2>&1 || { echo "TESTS FAILED $name" >> gpurun_out/tune.log; exit 1; }
  fi
  chk=--check; case "$name" in abl*) chk="";; esac   # ablation builds are timing-only (wrong results)
  GELLY_HIP_LIB="$PWD/$v/libgellyhip.so" timeout -k 10 300 python bench.py $chk --steps 8 --warmup 2 --no-cpu-baseline \
    > "gpurun_out/tune_$name.json" 2>> gpurun_out/tune.log || { echo "FAILED $name rc=$?" >> gpurun_out/tune.log; exit 1; }
done
