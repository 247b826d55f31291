#!/bin/bash
# Secondary workloads C1 / C5 (bench.py --workload c1|apply|candidates); every step time-limited.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 200 python bench.py --workload c1 --steps 10 --warmup 2 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err &&
timeout -k 10 300 python bench.py --workload apply --steps 10 --warmup 2 > gpurun_out/bench_apply.json 2> gpurun_out/bench_apply.err &&
timeout -k 10 300 python bench.py --workload candidates --steps 5 --warmup 1 > gpurun_out/bench_cand.json 2> gpurun_out/bench_cand.err &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 tools/exchange_timing.py > gpurun_out/exchange_timing.txt 2> gpurun_out/exchange_timing.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err
