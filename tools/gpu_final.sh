#!/bin/bash
# Round-end evidence on one GPU box, in three calls (each under gpurun's 1200 s limit):
#   bash tools/gpu_final.sh A TAG   the whole -m gpu suite, smoke(), the default bench line (with cpu_baseline)
#   bash tools/gpu_final.sh B TAG   C2 kernel trace + PMC traffic; triangles s24 / s26 trace + PMC
#   bash tools/gpu_final.sh C TAG   every secondary bench line DESIGN.md quotes (tools/gpu.sh evidence)
#   bash tools/gpu_final.sh D TAG   the opt-in C4 window parity test (R-MAT s26, 2^30 edges, GS_TEST_S26=1)
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
esac
