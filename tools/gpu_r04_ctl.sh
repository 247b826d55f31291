#!/bin/bash
# round 4: bench.py under torch.distributed.run (as the driver launches N > 1) at world 1, control plane
# nccl vs gloo (--control-pg), alternating, same box
# (the --control-pg switch lived in an A/B build of bench.py only; the kept bench uses the nccl process group)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04ctl}
mkdir -p $O
port=29540
r() { local name=$1; shift; port=$((port + 1)); timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" \
        > $O/$name.json 2> $O/$name.err; echo "$name done"; }
for i in 1 2; do
  r nccl_$i --control-pg nccl
  r gloo_$i --control-pg gloo
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/plain.json 2> $O/plain.err
echo plain done
