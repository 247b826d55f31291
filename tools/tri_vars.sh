#!/bin/bash
# bench several triangle build variants against the default at one scale.  GPU box, repo root.
#   bash tools/tri_vars.sh OUT SCALE VARIANT...
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; s=$2; shift 2
mkdir -p $O
st=10; [ $s -ge 26 ] && st=3
timeout -k 10 300 python bench.py --workload triangles --scale $s --steps $st --warmup 1 --no-cpu-baseline > $O/main.s$s.json 2>/dev/null
for V in "$@"; do
  GELLY_HIP_LIB=gelly-streaming_amd/variants/$V/libgellyhip.so timeout -k 10 300 python bench.py --workload triangles --scale $s --steps $st --warmup 1 --no-cpu-baseline > $O/$V.s$s.json 2>/dev/null
done
