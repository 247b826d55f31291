#!/bin/bash
# Kernel trace of the forced exchange at world size 1 (what each rank pays at N > 1): bench.py reads the
# torchrun variables itself, so rocprofv3 runs python directly (no launcher in between).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29514
O=gpurun_out/${1:-dist_trace}
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 bench.py --gpus 1 \
  --steps 5 --warmup 2 --exchange abi --force-exchange --no-cpu-baseline > "$O/forced.json" 2> "$O/forced.err"
echo trace done
