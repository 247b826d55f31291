#!/bin/bash
# round 4: is the heavy count bound by the items in flight?  TH_ILP 4 / 8 / 16 at s24 and s26; timing
# levels test + C2 bench with the lean timed region
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_bucket.py::test_timing_levels_same_results" tests/test_gpu_fresh_process.py > $O/tests.txt 2>&1
echo tests done
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/c2_dom_$i.json 2> $O/c2_dom_$i.err
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --timing stages > $O/c2_stages_$i.json 2> $O/c2_stages_$i.err
done
echo c2 done
for v in default ilp4 ilp16 hmin128 hmin64; do
  lib=""; [ $v = default ] || lib=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so
  for s in 24 26; do
    env ${lib:+GELLY_HIP_LIB=$lib} timeout -k 10 300 python3 bench.py --workload triangles --scale $s --steps 2 --warmup 1 \
      --no-cpu-baseline > $O/${v}_s$s.json 2> $O/${v}_s$s.err
    echo "$v s$s done"
  done
done
