#!/bin/bash
# WindowTriangles at growing R-MAT scales (C4 shape) + exchange timing + final default-bench profile
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python bench.py --workload triangles --scale 22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tri22.json 2> gpurun_out/bench_tri22.err &&
timeout -k 10 200 python bench.py --workload triangles --scale 24 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tri24.json 2> gpurun_out/bench_tri24.err &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 tools/exchange_timing.py > gpurun_out/exchange_timing.txt 2> gpurun_out/exchange_timing.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_final.log 2>&1
