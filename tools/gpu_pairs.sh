#!/bin/bash
# stage-2 candidate count: GPU tests + the candidates bench line (emission + stage 2)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_api.py -k "count_candidates or two_stage" > gpurun_out/pairs_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --workload candidates --steps 5 --warmup 1 > gpurun_out/bench_cand.json 2> gpurun_out/bench_cand.err
