#!/bin/bash
# Short GPU session: parity tests (bucket path first), the default bench line and the sort-path ablation.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_bucket.py -x -q -m gpu > gpurun_out/gpu_bucket.log 2>&1 &&
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --check > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --sort-only --no-cpu-baseline > gpurun_out/bench_sort.json 2> gpurun_out/bench_sort.err &&
timeout -k 10 300 python bench.py --workload fold --steps 5 --warmup 2 > gpurun_out/bench_fold.json 2> gpurun_out/bench_fold.err
