#!/bin/bash
# Round-end evidence on one GPU box, in three calls (each under gpurun's 1200 s limit):
#   bash tools/gpu_final.sh A TAG   the whole -m gpu suite, smoke(), the default bench line (with cpu_baseline)
#   bash tools/gpu_final.sh B TAG   C2 kernel trace + PMC traffic; triangles s24 / s26 trace + PMC
#   bash tools/gpu_final.sh C TAG   every secondary bench line DESIGN.md quotes (tools/gpu.sh evidence)
#   bash tools/gpu_final.sh D TAG   the opt-in C4 window parity test (R-MAT s26, 2^30 edges, GS_TEST_S26=1)
#   bash tools/gpu_final.sh E TAG   C5 lines with 32-bit and 64-bit id columns (cpu_baseline) + an emission kernel trace
#   bash tools/gpu_final.sh F TAG   round 6: C2 evidence (line, trace, PMC, write attribution, timeline, atomics microbench)
#   bash tools/gpu_final.sh G TAG   round 6: secondary lines (Double, C3, CC, C1, apply, candidates, parse, e2e)
#   bash tools/gpu_final.sh H TAG   round 6: triangles s20-s26 (s26 with the whole-window CPU baseline), C5 lines
#   bash tools/gpu_final.sh I TAG   round 6, last build: C2 line + trace + PMC traffic; triangles s26 line (whole-window
#                                   CPU baseline) + trace + FETCH / SQ passes; s20 / s22 / s24 lines
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
  F)   # round 6: the C2 headline's evidence (bench line, kernel trace, PMC traffic, write attribution, the window
       # timeline and its gaps, the no-partition atomic microbench)
    bash tools/gpu.sh c2 "$TAG"
    bash tools/gpu.sh wr "$TAG"
    bash tools/gpu.sh c2trace "$TAG" --steps 10 --warmup 3
    timeout -k 10 120 ./tools/microbench/global_atomic > "$O/no_partition_atomics.json" 2> "$O/no_partition_atomics.err" ;;
  G)   # round 6: secondary lines without triangles / C5
    for x in "bench_c2_f64 --dtype float64" "bench_c3_rmat --workload fold" "bench_c3_zipf --workload fold --stream zipf" \
             "bench_cc_s24 --workload cc" "bench_c1 --workload c1" "bench_apply --workload apply" \
             "bench_candidates --workload candidates" "bench_parse --workload parse" \
             "bench_e2e_direct --workload e2e --staging direct --no-cpu-baseline" \
             "bench_e2e_pinned --workload e2e --staging pinned --no-cpu-baseline"; do
      set -- $x; n=$1; shift
      timeout -k 10 300 python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err"; echo "$n done"
    done ;;
  H)   # round 6: triangles (s20 / s22 / s24 lines; s26 with the whole-window 16-thread CPU baseline) and C5
    for x in "bench_tri_s20 --workload triangles --scale 20" "bench_tri_s22 --workload triangles --scale 22" \
             "bench_tri_s24 --workload triangles --scale 24"; do
      set -- $x; n=$1; shift
      timeout -k 10 300 python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err"; echo "$n done"
    done
    timeout -k 10 400 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 > "$O/bench_tri_s26.json" 2> "$O/bench_tri_s26.err"
    echo "bench_tri_s26 done"
    timeout -k 10 300 python3 bench.py --workload cand_stream --cand-windows 4 > "$O/bench_cand_stream.json" 2> "$O/bench_cand_stream.err"
    timeout -k 10 300 python3 bench.py --workload cand_stream --cand-windows 4 --cand-ids u32 > "$O/bench_cand_stream_u32.json" 2> "$O/bench_cand_stream_u32.err"
    timeout -k 10 300 python3 bench.py --workload cand_stream --cand-windows 4 --cand-cadence-ms 1000 --no-cpu-baseline > "$O/bench_cand_stream_cadence.json" 2> "$O/bench_cand_stream_cadence.err" ;;
  I)
    bash tools/gpu.sh c2 "$TAG"
    bash tools/gpu.sh tri "$TAG" 26
    for x in "bench_tri_s20 --workload triangles --scale 20" "bench_tri_s22 --workload triangles --scale 22" \
             "bench_tri_s24 --workload triangles --scale 24"; do
      set -- $x; n=$1; shift
      timeout -k 10 300 python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err"; echo "$n done"
    done ;;
  E)
    timeout -k 10 400 python3 bench.py --workload cand_stream --cand-ids u32 > "$O/bench_cand_stream_u32.json" 2> "$O/bench_cand_stream_u32.err"
    timeout -k 10 400 python3 bench.py --workload cand_stream > "$O/bench_cand_stream.json" 2> "$O/bench_cand_stream.err"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/cand_u32_trace" -o run --output-format csv -- python3 bench.py --workload cand_stream \
      --cand-ids u32 --cand-consumer none --cand-windows 1 --max-chunks 40 --no-cpu-baseline > "$O/cand_u32_trace.log" 2>&1 ;;
esac
