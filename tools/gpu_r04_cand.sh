#!/bin/bash
# round 4: candidate emission rewrite -- parity tests, then the C5 stream bench and its kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -rP \
  tests/test_gpu_candidates_chunked.py tests/test_gpu_fresh_process.py tests/test_gpu_api.py tests/test_gpu_dist.py \
  "tests/test_gpu_config_size.py::test_c5_window_candidate_records_vertex_ranges" \
  "tests/test_gpu_config_size.py::test_c5_window_candidate_count_vs_oracle" > gpurun_out/r04_cand_tests.log 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --workload cand_stream > gpurun_out/r04_cand_stream.json 2> gpurun_out/r04_cand_stream.err || exit 2
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cand" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload cand_stream > "$GRAFT_REPO_ROOT/gpurun_out/r04_cand_prof.log" 2>&1 || exit 3
