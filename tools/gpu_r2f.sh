#!/bin/bash
# Round 2, pass f: triangle kernels (long-list gathers) — tests + s20/s22/s24 benches vs previous
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_config_size.py -v -m gpu -k "tri or c4 or clique or cand" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_f.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for s in 20 22 24; do
  timeout -k 10 300 python bench.py --workload triangles --scale $s --steps 5 --warmup 2 --no-cpu-baseline --windows 1 > gpurun_out/tri_f_s$s.json 2> gpurun_out/tri_f_s$s.err || exit 1
done
