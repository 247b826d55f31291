#!/bin/bash
# A/B of triangle-count tuning builds (GELLY_HIP_LIB) at scales 22 and 24: main + the listed variants
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab_tri
export TMPDIR=/tmp
for v in main "$@"; do
  for s in 22 24; do
    if [ "$v" = main ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
    GELLY_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload triangles --scale $s --steps 5 --warmup 2 --no-cpu-baseline --windows 1 > gpurun_out/ab_tri/$v.s$s.json 2> gpurun_out/ab_tri/$v.s$s.err || exit 1
  done
done
