#!/bin/bash
# Round 2, pass b: dist ABI tests, packed tests, scatter variants A/B, torchrun world 1
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_bucket.py tests/test_gpu_api.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for v in pk4 it8; do
  GELLY_HIP_LIB=gelly-streaming_amd/variants/$v/libgellyhip.so timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/bench_main.json 2> gpurun_out/bench_main.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err
