#!/bin/bash
# round 4: candidate emission -- batched id gathers (in-tree), register caps for 6 / 8 waves per SIMD
# (variants/ce6, ce8) and the previous build (variants/pre) on the whole C5 window
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04e2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_candidates_chunked.py \
  "tests/test_gpu_config_size.py::test_c5_window_candidate_records_vertex_ranges" > $O/tests.txt 2>&1
for v in ce6 ce8; do
  GELLY_HIP_LIB=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 600 \
    --timeout-method thread -m gpu tests/test_gpu_candidates_chunked.py > $O/tests_$v.txt 2>&1
done
echo tests done
for i in 1 2; do
  for v in default pre ce6 ce8; do
    lib=""; [ $v = default ] || lib=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so
    env ${lib:+GELLY_HIP_LIB=$lib} timeout -k 10 240 python3 bench.py --workload cand_stream --no-cpu-baseline \
      > $O/${v}_$i.json 2> $O/${v}_$i.err
  done
  echo "round $i done"
done
