#!/bin/bash
# Round 2, pass r: the cc and triangle bench lines (after pass q)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r2q
export TMPDIR=/tmp
B="timeout -k 10 300 python bench.py"
$B --workload cc --steps 5 --warmup 2 > gpurun_out/r2q/cc_s24.json 2> gpurun_out/r2q/cc_s24.err || exit 1
$B --workload triangles --scale 24 --steps 4 --warmup 1 > gpurun_out/r2q/tri_s24.json 2> gpurun_out/r2q/tri_s24.err || exit 1
