#!/bin/bash
# round 4: candidate emission with the slot metadata cached across steps -- chunked candidate tests, then
# cand_stream (whole C5 window) against the previous build (variants/pre)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_candidates_chunked.py \
  "tests/test_gpu_config_size.py::test_c5_window_candidate_records_vertex_ranges" > $O/tests.txt 2>&1
echo tests done
pre=$PWD/gelly-streaming_amd/variants/pre/libgellyhip.so
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --workload cand_stream --no-cpu-baseline > $O/new_$i.json 2> $O/new_$i.err
  GELLY_HIP_LIB=$pre timeout -k 10 240 python3 bench.py --workload cand_stream --no-cpu-baseline > $O/pre_$i.json 2> $O/pre_$i.err
  echo "round $i done"
done
