#!/bin/bash
# full GPU suite + plain vs torchrun (world 1) bench lines in one session
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err &&
timeout -k 10 300 python bench.py --workload fold --steps 10 --warmup 3 > gpurun_out/bench_fold.json 2> gpurun_out/bench_fold.err
