#!/bin/bash
# GPU session: the bucket-path parity tests, the bench line (+ CPU baseline), the onesweep A/B line,
# rocprofv3 kernel-trace + FETCH_SIZE / WRITE_SIZE passes of the bench, and the whole GPU suite.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline"
P=gpurun_out/prof_direct
timeout -k 10 600 $T tests/test_gpu_bucket.py -m gpu > gpurun_out/gpu_bucket.log 2>&1 &&
timeout -k 10 300 python bench.py --check > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --bk-onesweep --no-cpu-baseline > gpurun_out/bench_os.json 2> gpurun_out/bench_os.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $B > $P.trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python3 $B > $P.fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python3 $B > $P.write.log 2>&1 &&
timeout -k 10 900 $T tests/ -m gpu > gpurun_out/gpu_tests.log 2>&1
