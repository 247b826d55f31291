#!/bin/bash
# A/B of triangle tuning builds at scale 26 (the C4 window): main + the listed variants
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab_tri
export TMPDIR=/tmp
for v in main "$@"; do
  if [ "$v" = main ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
  GELLY_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload triangles --scale 26 --steps 2 --warmup 1 --no-cpu-baseline --windows 1 > gpurun_out/ab_tri/$v.s26.json 2> gpurun_out/ab_tri/$v.s26.err || exit 1
done
