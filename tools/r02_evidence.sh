#!/bin/bash
# Round-2 evidence refresh: every bench line DESIGN.md quotes, plus rocprofv3 kernel stats of the C2
# headline and the s24 triangle window.  GPU box, repo root:  bash tools/r02_evidence.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ev}
mkdir -p $O
b() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b bench_c2_i64
b bench_c2_f64 --dtype float64
b bench_c3_rmat --workload fold
b bench_c3_zipf --workload fold --stream zipf
b bench_tri_s20 --workload triangles --scale 20
b bench_tri_s22 --workload triangles --scale 22
b bench_tri_s24 --workload triangles --scale 24
b bench_tri_s26 --workload triangles --scale 26 --steps 3 --warmup 1
b bench_cc_s24 --workload cc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace_c2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_tri24 -o run --output-format csv -- python3 bench.py --workload triangles --scale 24 --steps 3 --warmup 1 --no-cpu-baseline > $O/trace_tri24.log 2>&1
echo all done
