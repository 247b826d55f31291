#!/bin/bash
# Counter passes over a short C2 bench (the first window takes the histogram path, the rest the
# speculative one, so both scatter kernels appear).  Run on the GPU box from the repo root.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmc_sc
mkdir -p $O
run() {   # name, counters
  timeout -s KILL 150 rocprofv3 --pmc $2 -d $O/$1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/$1.log 2>&1
}
run sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
run sq2 "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
python3 tools/pmc_summary.py $O/sq $O/sq2 $O/fetch $O/write > $O/summary.txt 2>&1 || true
