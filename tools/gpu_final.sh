#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke(), default bench line, torchrun world-1 line, rocprof trace
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_final.log 2>&1 &&
timeout -k 10 300 python bench.py --workload fold --steps 10 --warmup 3 > gpurun_out/bench_fold.json 2> gpurun_out/bench_fold.err &&
timeout -k 10 200 python bench.py --workload c1 --steps 10 --warmup 2 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err &&
timeout -k 10 200 python bench.py --workload triangles --scale 20 --steps 5 --warmup 2 > gpurun_out/bench_tri.json 2> gpurun_out/bench_tri.err
