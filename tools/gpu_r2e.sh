#!/bin/bash
# Round 2, pass e: stream operator + relabel tests, e2e bench (direct / pinned staging)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread --ignore=tests/test_gpu_config_size.py > gpurun_out/gpu_tests_e.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload e2e --steps 4 --warmup 2 --check --staging direct > gpurun_out/bench_e2e_direct.json 2> gpurun_out/bench_e2e_direct.err || exit 1
timeout -k 10 400 python bench.py --workload e2e --steps 4 --warmup 2 --check --staging pinned > gpurun_out/bench_e2e_pinned.json 2> gpurun_out/bench_e2e_pinned.err
