#!/bin/bash
# rocprofv3 kernel-trace + separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) over a short bench.
# Usage: tools/profile.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/...
cd "$(dirname "$0")/.." || exit 1
tag=$1; shift
out=$PWD/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
B="$PWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 $B > "$out/trace.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 $B > "$out/fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 $B > "$out/write.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$out/sq1" -o run --output-format csv -- python3 $B > "$out/sq1.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d "$out/sq2" -o run --output-format csv -- python3 $B > "$out/sq2.log" 2>&1 || exit 1
