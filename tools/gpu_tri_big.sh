#!/bin/bash
# WindowTriangles at R-MAT s25 and s26 (the C4 window, here on one GPU); each step time-limited
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 240 python -u bench.py --workload triangles --scale 25 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tri25.json 2> gpurun_out/bench_tri25.err &&
timeout -k 10 400 python -u bench.py --workload triangles --scale 26 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tri26.json 2> gpurun_out/bench_tri26.err
