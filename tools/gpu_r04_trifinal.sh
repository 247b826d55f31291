#!/bin/bash
# round 4: triangle bench lines s20-s24 and the s26 bench + kernel trace + PMC passes on the final build
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04trifinal}
mkdir -p $O
for s in 20 22 24; do
  timeout -k 10 300 python3 bench.py --workload triangles --scale $s > $O/bench_tri_s$s.json 2> $O/bench_tri_s$s.err
  echo "s$s done"
done
bash tools/gpu.sh tri ${1:-r04trifinal} 26
