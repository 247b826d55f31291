#!/bin/bash
# Round 2, pass u: exact JDK HashSet order on the GPU (tests), s26 A/B of the hw8 tuning, C5-shape e2e
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -v -m gpu -k "cand or jdk or self_loops or arbitrary" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_u.log 2>&1 || exit $?
bash tools/ab_tri26.sh hw8 hlw8i6 || exit $?
timeout -k 10 500 python bench.py --workload e2e --e2e-kind triangles --scale 23 --windows-edges 1e8 --steps 5 --warmup 2 > gpurun_out/e2e_c5_u.json 2> gpurun_out/e2e_c5_u.err
