#!/bin/bash
# HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE in separate rocprofv3 passes) for the C2 bench,
# speculative partition vs per-tile histograms.  Run on the GPU box from the repo root.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_ab
for mode in spec nospec; do
  extra=""
  [ "$mode" = nospec ] && extra="--no-spec"
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/$mode/$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 150 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline $extra > $O.$mode.$c.log 2>&1
  done
  python3 tools/pmc_traffic.py $O/$mode -o $O/$mode.json
done
