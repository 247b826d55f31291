#!/bin/bash
# A/B of the host wait (polled event vs blocking stream sync), plain and under torchrun, repeated
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline"
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551"
for i in 1 2; do
  timeout -k 10 200 python $B > gpurun_out/ab/plain_poll_$i.json 2>/dev/null || exit 1
  GS_BLOCKING_WAIT=1 timeout -k 10 200 python $B > gpurun_out/ab/plain_block_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 $TR $B --gpus 1 > gpurun_out/ab/tr_poll_$i.json 2>/dev/null || exit 1
  GS_BLOCKING_WAIT=1 timeout -k 10 200 $TR $B --gpus 1 > gpurun_out/ab/tr_block_$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py > gpurun_out/ab/default_poll.json 2>/dev/null || exit 1
GS_BLOCKING_WAIT=1 timeout -k 10 300 python bench.py > gpurun_out/ab/default_block.json 2>/dev/null
