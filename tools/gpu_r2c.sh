#!/bin/bash
# Round 2, pass c: packed-scatter tile A/B (items per thread, blocks per CU)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ab_main.json 2> gpurun_out/ab_main.err || exit 1
for v in pki12 pki14 pki16 pk8w; do
  GELLY_HIP_LIB=gelly-streaming_amd/variants/$v/libgellyhip.so timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
done
GELLY_HIP_LIB=gelly-streaming_amd/variants/pki16/libgellyhip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_parity.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pki16_tests.log 2>&1
