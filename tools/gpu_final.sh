#!/bin/bash
# Round-end evidence on one GPU box, in three calls (each under gpurun's 1200 s limit):
#   bash tools/gpu_final.sh A TAG   the whole -m gpu suite, smoke(), the default bench line (with cpu_baseline)
#   bash tools/gpu_final.sh B TAG   C2 kernel trace + PMC traffic; triangles s24 / s26 trace + PMC
#   bash tools/gpu_final.sh C TAG   every secondary bench line DESIGN.md quotes (tools/gpu.sh evidence)
#   bash tools/gpu_final.sh D TAG   the opt-in C4 window parity test (R-MAT s26, 2^30 edges, GS_TEST_S26=1)
#   bash tools/gpu_final.sh E TAG   C5 lines with 32-bit and 64-bit id columns (cpu_baseline) + an emission kernel trace
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
MODE=$1; TAG=${2:-final}
O=gpurun_out/$TAG
mkdir -p "$O"
case $MODE in
  A)
    bash tools/gpu.sh tests "$TAG"
    tail -3 "$O/tests.txt"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
    cat "$O/smoke.txt" | grep -v amdgpu.ids
    bash tools/gpu.sh bench "$TAG" ;;
  B)
    bash tools/gpu.sh c2 "$TAG"
    bash tools/gpu.sh tri "$TAG" 24
    bash tools/gpu.sh tri "$TAG" 26 ;;
  C)
    bash tools/gpu.sh evidence "$TAG" ;;
  D)
    GS_TEST_S26=1 timeout -k 10 1100 python -u -m pytest -x -v --timeout 1000 --timeout-method thread -m gpu \
      tests/test_gpu_config_size.py -k s26 > "$O/tests_s26.txt" 2>&1
    tail -3 "$O/tests_s26.txt" ;;
  E)
    timeout -k 10 400 python3 bench.py --workload cand_stream --cand-ids u32 > "$O/bench_cand_stream_u32.json" 2> "$O/bench_cand_stream_u32.err"
    timeout -k 10 400 python3 bench.py --workload cand_stream > "$O/bench_cand_stream.json" 2> "$O/bench_cand_stream.err"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/cand_u32_trace" -o run --output-format csv -- python3 bench.py --workload cand_stream \
      --cand-ids u32 --cand-consumer none --cand-windows 1 --max-chunks 40 --no-cpu-baseline > "$O/cand_u32_trace.log" 2>&1 ;;
esac
