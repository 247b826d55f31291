#!/bin/bash
# Short GPU session: the bucket-path parity tests, then the default bench line (+ optional extra bench args).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bucket.py -m gpu > gpurun_out/gpu_bucket.log 2>&1 &&
timeout -k 10 300 python bench.py --check "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
