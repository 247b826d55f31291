#!/bin/bash
# Round 2, first GPU pass: fast GPU suite, C2 bench (packed vs unpacked), config-size parity, rocprof trace
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -v -m gpu --timeout 120 --timeout-method thread \
    --ignore=tests/test_gpu_config_size.py > gpurun_out/gpu_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc   # test failures: go on; a crash / timeout: stop here
timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-pack --no-cpu-baseline > gpurun_out/bench_nopack.json 2> gpurun_out/bench_nopack.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests/test_gpu_config_size.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_config_tests.log 2>&1
