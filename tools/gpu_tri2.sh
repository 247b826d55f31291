#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_api.py -k "triangle or parts" > gpurun_out/tri2_tests.log 2>&1 &&
timeout -k 10 120 python bench.py --workload triangles --scale 20 --steps 5 --warmup 2 > gpurun_out/tri2_s20.json 2> gpurun_out/tri2_s20.err &&
timeout -k 10 120 python bench.py --workload triangles --scale 22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tri2_s22.json 2> gpurun_out/tri2_s22.err &&
timeout -k 10 200 python bench.py --workload triangles --scale 24 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tri2_s24.json 2> gpurun_out/tri2_s24.err &&
timeout -k 10 400 python bench.py --workload triangles --scale 26 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tri2_s26.json 2> gpurun_out/tri2_s26.err
