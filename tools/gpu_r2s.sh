#!/bin/bash
# Round 2, pass s: connected components with direct ids: tests + the cc line
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r2q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_components.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2q/cc_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload cc --steps 5 --warmup 2 > gpurun_out/r2q/cc_s24.json 2> gpurun_out/r2q/cc_s24.err || exit 1
