#!/bin/bash
# Triangle tests + bench A/B of the heavy-kernel bitmap (variant nobm = GS_TH_BITMAP=0).  GPU box, repo root.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tri_ab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_config_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tri or Tri" > $O/tests.txt 2>&1
for s in 22 24; do
  timeout -k 10 200 python bench.py --workload triangles --scale $s --no-cpu-baseline > $O/bm.s$s.json 2>/dev/null
  GELLY_HIP_LIB=gelly-streaming_amd/variants/nobm/libgellyhip.so timeout -k 10 200 python bench.py --workload triangles --scale $s --no-cpu-baseline > $O/nobm.s$s.json 2>/dev/null
done
timeout -k 10 300 python bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/bm.s26.json 2>/dev/null
