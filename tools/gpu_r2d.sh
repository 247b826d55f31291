#!/bin/bash
# Round 2, pass d: full GPU suite, C2 bench + rocprof trace + PMC traffic passes, e2e stream bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_d.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --check > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err || exit 1
out=gpurun_out/prof_d
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $B > $out.trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 $B > $out.fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 $B > $out.write.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload e2e --steps 4 --warmup 2 --check > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err
