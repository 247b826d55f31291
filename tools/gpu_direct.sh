#!/bin/bash
# GPU session for the direct bucket partition: its parity tests first, then the bench line, the
# onesweep A/B line, a rocprofv3 kernel-trace of the bench, and the whole GPU suite.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_bucket.py -m gpu > gpurun_out/gpu_bucket.log 2>&1 &&
timeout -k 10 300 python bench.py --check > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --bk-onesweep --no-cpu-baseline > gpurun_out/bench_os.json 2> gpurun_out/bench_os.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_direct -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_direct.log 2>&1 &&
timeout -k 10 900 $T tests/ -m gpu > gpurun_out/gpu_tests.log 2>&1
