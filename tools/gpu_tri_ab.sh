#!/bin/bash
# A/B of triangle tuning builds (gelly-streaming_amd/variants/*) at R-MAT s24 and s26, plus the in-tree build
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tri_ab
for v in default gelly-streaming_amd/variants/*/; do
  name=$(basename "$v")
  lib=""; [ "$v" = default ] || lib="$PWD/$v/libgellyhip.so"
  for s in 24 26; do
    env ${lib:+GELLY_HIP_LIB=$lib} timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 2 --warmup 1 \
      --no-cpu-baseline > gpurun_out/tri_ab/${name}_s$s.json 2>> gpurun_out/tri_ab/log.txt
    echo "$name s$s done"
  done
done
