#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 tools/exchange_timing.py > gpurun_out/exchange_timing.txt 2> gpurun_out/exchange_timing.err
