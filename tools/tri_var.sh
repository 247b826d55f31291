#!/bin/bash
# bench a triangle build variant against the default at the given scales.  GPU box, repo root.
#   bash tools/tri_var.sh OUT VARIANT SCALE...
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; V=$2; shift 2
mkdir -p $O
for s in "$@"; do
  st=10; [ $s -ge 26 ] && st=3
  timeout -k 10 300 python bench.py --workload triangles --scale $s --steps $st --warmup 1 --no-cpu-baseline > $O/main.s$s.json 2>/dev/null
  GELLY_HIP_LIB=gelly-streaming_amd/variants/$V/libgellyhip.so timeout -k 10 300 python bench.py --workload triangles --scale $s --steps $st --warmup 1 --no-cpu-baseline > $O/$V.s$s.json 2>/dev/null
done
