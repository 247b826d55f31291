#!/bin/bash
# round 4: emission fast path (tests + C5 stream + trace), triangles s26 okeys split A/B, C2 default line
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -rP \
  tests/test_gpu_candidates_chunked.py "tests/test_gpu_api.py" \
  "tests/test_gpu_config_size.py::test_c5_window_candidate_records_vertex_ranges" > $O/tests.txt 2>&1
echo tests done
timeout -k 10 240 python3 bench.py --workload cand_stream > $O/cand_stream.json 2> $O/cand_stream.err
echo cand_stream done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/trace_cand" -o run --output-format csv \
  -- python3 bench.py --workload cand_stream > $O/trace_cand.log 2>&1
echo trace done
timeout -k 10 400 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/tri_s26_split.json 2> $O/tri_s26_split.err
echo tri split done
GS_TRI_OKEYS_SPLIT=0 timeout -k 10 400 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/tri_s26_nosplit.json 2> $O/tri_s26_nosplit.err
echo tri nosplit done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
echo all done
