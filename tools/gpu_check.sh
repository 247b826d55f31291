#!/bin/bash
# One GPU session: parity tests, the default bench line, the torchrun/RCCL path at world 1, and the
# secondary workloads.  Every GPU step has its own time limit; the chain stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --check > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err &&
timeout -k 10 300 python bench.py --workload fold --steps 5 --warmup 2 > gpurun_out/bench_fold.json 2> gpurun_out/bench_fold.err &&
timeout -k 10 300 python bench.py --workload triangles --scale 20 --steps 3 --warmup 1 > gpurun_out/bench_tri.json 2> gpurun_out/bench_tri.err
