#!/bin/bash
# PMC passes over the s22 triangle bench (one counter group per run)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/pmc_tri
export TMPDIR=/tmp
B="bench.py --workload triangles --scale 22 --steps 1 --warmup 0 --no-cpu-baseline --windows 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_tri/sq -o run --output-format csv -- python3 $B > gpurun_out/pmc_tri/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD -d gpurun_out/pmc_tri/sq2 -o run --output-format csv -- python3 $B > gpurun_out/pmc_tri/sq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_tri/ta -o run --output-format csv -- python3 $B > gpurun_out/pmc_tri/ta.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/pmc_tri/fetch -o run --output-format csv -- python3 $B > gpurun_out/pmc_tri/fetch.log 2>&1
