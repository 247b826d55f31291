#!/bin/bash
# per-kernel trace of one triangles bench (rocprofv3 --kernel-trace --stats), scale $1 (default 22)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${1:-22}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tri_s$S -o run --output-format csv -- python3 bench.py --workload triangles --scale $S --steps 3 --warmup 1 --no-cpu-baseline --windows 1 > gpurun_out/prof_tri_s$S.log 2>&1
