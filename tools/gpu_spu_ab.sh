#!/bin/bash
# A/B of the unpacked speculative scatter's tile (gelly-streaming_amd/variants/*): C3 R-MAT / Zipf, Double C2
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/spu_ab
for v in default gelly-streaming_amd/variants/*/; do
  name=$(basename "$v"); lib=""; [ "$v" = default ] || lib="$PWD/$v/libgellyhip.so"
  for w in "c3_rmat --workload fold" "c3_zipf --workload fold --stream zipf" "c2_f64 --dtype float64"; do
    set -- $w; t=$1; shift
    env ${lib:+GELLY_HIP_LIB=$lib} timeout -k 10 300 python3 bench.py "$@" --steps 8 --no-cpu-baseline \
      > gpurun_out/spu_ab/${name}_$t.json 2>/dev/null
  done
  echo "$name done"
done
