#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/pmc_parse
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_parse -o run --output-format csv -- python3 bench.py --workload parse --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_parse/log.txt 2>&1
