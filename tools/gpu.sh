#!/bin/bash
# The one GPU-box launcher (run from the repo root, under gpurun):  bash tools/gpu.sh MODE [TAG] [ARGS...]
#
#   tests   TAG [pytest args]   the -m gpu suite (default: all of tests/), log in gpurun_out/TAG/tests.txt
#   bench   TAG [bench args]    one bench.py line -> gpurun_out/TAG/bench.json
#   c2      TAG                 the C2 headline: bench line (+ cpu_baseline), rocprofv3 kernel-trace stats of
#                               the same command, FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json
#   c2pmc   TAG                 only the FETCH_SIZE / WRITE_SIZE passes of c2
#   sq      TAG [bench args]    SQ counter passes (LDS conflicts, waits, instruction mix) over a short bench
#   tri     TAG SCALE           triangles: bench line, kernel-trace stats, FETCH / TCC hit / SQ passes
#   evidence TAG                every secondary bench line DESIGN.md quotes
#   ttrace  TAG SCALE           triangles: the kernel trace alone
#   ktrace  TAG NAME [args]     the kernel trace of any bench line
#   envab   TAG "base K=V .." [args] A/B of environment knobs, alternated twice on one box
#   ab      TAG "V1 V2.." [args] A/B of tuning builds (csrc/Makefile bvariant / variant -> variants/NAME; "base" =
#                               the in-tree library): bench lines alternated twice on one box -> ab_NAME_REP.json
#
# Every GPU step has its own time limit and the chain stops at the first failure (set -e): after a
# fault, an abort or a timeout nothing more runs on the GPU in that call.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
MODE=$1; TAG=${2:-run}; shift 2 || true
O=gpurun_out/$TAG
mkdir -p "$O"
PYTEST="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
bench() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > "$O/$name.json" 2> "$O/$name.err"; echo "$name done"; }
trace() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv \
            -- python3 bench.py "$@" --no-cpu-baseline > "$O/$name.log" 2>&1; echo "$name done"; }
pmc() { local name=$1 counters=$2; shift 2; mkdir -p "$(dirname "$O/$name")"; timeout -s KILL 150 rocprofv3 --pmc $counters -d "$O/$name" -o run \
          --output-format csv -- python3 bench.py "$@" --no-cpu-baseline > "$O/$name.log" 2>&1; echo "$name done"; }

case $MODE in
  tests)
    [ $# -gt 0 ] || set -- tests/
    timeout -k 10 1000 $PYTEST -m gpu "$@" > "$O/tests.txt" 2>&1 ;;
  bench)
    bench bench "$@" ;;
  c2)
    bench bench_c2_i64
    trace trace_c2
    ;&
  c2pmc)
    pmc pmc/fetch FETCH_SIZE --steps 3 --warmup 2
    pmc pmc/write WRITE_SIZE --steps 3 --warmup 2
    python3 tools/pmc_traffic.py "$O/pmc" -o "$O/pmc_traffic.json" ;;
  sq)
    pmc sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES" --steps 3 --warmup 2 "$@"
    pmc sq2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES" --steps 3 --warmup 2 "$@" ;;
  tri)
    S=${1:-24}; shift || true
    A="--workload triangles --scale $S --steps 3 --warmup 1"
    bench bench_tri_s$S $A
    trace trace_tri_s$S $A
    pmc pmc_tri_s$S/fetch "FETCH_SIZE TCC_HIT_sum" $A --windows 1
    pmc pmc_tri_s$S/sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" $A --windows 1 ;;
  ab)
    VARIANTS=$1; shift
    for rep in 1 2; do
      for v in $VARIANTS; do
        if [ "$v" = base ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
        GELLY_HIP_LIB=$lib bench ab_${v}_$rep "$@" --no-cpu-baseline
      done
    done ;;
  evidence)
    bench bench_c2_f64 --dtype float64
    bench bench_c3_rmat --workload fold
    bench bench_c3_zipf --workload fold --stream zipf
    bench bench_tri_s20 --workload triangles --scale 20
    bench bench_tri_s22 --workload triangles --scale 22
    bench bench_tri_s24 --workload triangles --scale 24
    bench bench_tri_s26 --workload triangles --scale 26 --steps 3 --warmup 1
    bench bench_cc_s24 --workload cc
    bench bench_c1 --workload c1
    bench bench_apply --workload apply
    bench bench_candidates --workload candidates
    bench bench_cand_stream --workload cand_stream
    bench bench_parse --workload parse
    bench bench_e2e_direct --workload e2e --staging direct --no-cpu-baseline
    bench bench_e2e_pinned --workload e2e --staging pinned --no-cpu-baseline
    bench bench_e2e_buffered --workload e2e --staging buffered --no-cpu-baseline ;;
  tapmc)
    # texture-address / L1 counters of the triangle count (why its scattered loads are or are not the bound)
    S=${1:-24}; shift || true
    A="--workload triangles --scale $S --steps 1 --warmup 0 --windows 1"
    pmc tapmc_s$S/ta "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" $A
    pmc tapmc_s$S/tcp "TCP_TCC_READ_REQ_sum TCP_TOTAL_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum" $A ;;
  ktrace)
    # kernel trace of any bench line: TAG NAME [bench args]
    N=${1:-run}; shift || true
    trace "trace_$N" "$@" ;;
  ttrace)
    # kernel trace of one triangle window size only: TAG SCALE
    S=${1:-24}; shift || true
    trace trace_tri_s$S --workload triangles --scale $S --steps 3 --warmup 1 "$@" ;;
  envab)
    # A/B of library knobs read from the environment ("base" = none; e.g. "base GS_TRI_OKEYS_PART=0"),
    # alternated twice on one box -> ab_NAME_REP.json
    VARIANTS=$1; shift
    for rep in 1 2; do
      for v in $VARIANTS; do
        if [ "$v" = base ]; then bench ab_base_$rep "$@" --no-cpu-baseline
        else ( export "$v"; bench "ab_${v//=/_}_$rep" "$@" --no-cpu-baseline ); fi
      done
    done ;;
  syncab)
    # A/B of GS_FLAG_ASYNC_OUTPUT (default) against calls that wait for their outputs, alternated twice
    for rep in 1 2; do
      bench ab_async_$rep --no-cpu-baseline "$@"
      bench ab_sync_$rep --no-cpu-baseline --sync-outputs "$@"
    done ;;
  c2trace)
    # the C2 window's kernel timeline (gaps between kernels and between windows), from a kernel trace
    trace trace_c2 "$@"
    python3 tools/timeline.py "$(find "$O/trace_c2" -name '*kernel_trace.csv' | head -1)" k_sp_scatter_pack 3 > "$O/c2_timeline.txt"
    python3 tools/window_gaps.py "$(find "$O/trace_c2" -name '*kernel_trace.csv' | head -1)" > "$O/c2_window_gaps.txt" ;;
  counters)
    timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1 ;;
  wr)
    # where a kernel's WRITE_SIZE comes from: 64-byte vs other write requests and atomics at the fabric
    pmc pmc_wr/a "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum" --steps 3 --warmup 2 "$@"
    pmc pmc_wr/b "WRITE_SIZE" --steps 3 --warmup 2 "$@" ;;
  *)
    echo "usage: tools/gpu.sh tests|bench|c2|sq|tri|evidence|counters|wr TAG [args]" >&2; exit 2 ;;
esac
echo "$MODE done"
