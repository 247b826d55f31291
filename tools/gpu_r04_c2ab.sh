#!/bin/bash
# round 4: C2 per-window event records A/B (variants/noev: GS_STAGE_EVENTS=0), alternating runs
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04c2
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/base_$i.json 2> $O/base_$i.err
  GELLY_HIP_LIB=$PWD/gelly-streaming_amd/variants/noev/libgellyhip.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 \
    --no-cpu-baseline > $O/noev_$i.json 2> $O/noev_$i.err
  echo "round $i done"
done
