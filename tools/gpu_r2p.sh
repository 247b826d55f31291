#!/bin/bash
# Round 2, pass p: split-window triangles (gs_tri_dist_*), part slices — tests + s20/s22/s24 benches vs previous
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_config_size.py tests/test_gpu_stream.py tests/test_gpu_dist.py -v -m gpu -k "tri or c4 or clique or cand or part" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_p.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for s in 20 22 24; do
  timeout -k 10 300 python bench.py --workload triangles --scale $s --steps 5 --warmup 2 --no-cpu-baseline --windows 1 > gpurun_out/tri_p_s$s.json 2> gpurun_out/tri_p_s$s.err || exit 1
done
