#!/bin/bash
# edge text parser: GPU tests + bench line + kernel trace
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_api.py -k "parse_edges or itcase" > gpurun_out/text_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --workload parse --steps 5 --warmup 2 > gpurun_out/bench_parse.json 2> gpurun_out/bench_parse.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_parse -o run --output-format csv -- python3 bench.py --workload parse --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_parse.log 2>&1
