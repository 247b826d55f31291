#!/bin/bash
# WindowTriangles: parity tests + one bench line (argument: tag)
set -o pipefail
tag=${1:-triq}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_api.py -k triangle > gpurun_out/${tag}_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload triangles --scale 20 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
