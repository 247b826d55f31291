#!/bin/bash
# round 4: C2 variants -- non-temporal column loads in the scatter (GS_SPK_NT) and 8 x 16-byte loads per lane
# in the accumulate (GS_BK_UNROLL=16), alternating with the in-tree build
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04c2v
mkdir -p $O
for i in 1 2 3; do
  for v in default spknt acc16; do
    lib=""; [ $v = default ] || lib=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so
    env ${lib:+GELLY_HIP_LIB=$lib} timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      > $O/${v}_$i.json 2> $O/${v}_$i.err
  done
  echo "round $i done"
done
