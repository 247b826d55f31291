#!/bin/bash
# Round-2 evidence, second refresh: triangle windows after the split change, the secondary workloads
# (C1, C5 apply / candidates, text parse, end-to-end lines) and kernel stats of the s26 window.
# GPU box, repo root:  bash tools/r02_evidence2.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-ev2}
mkdir -p $O
b() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b bench_tri_s20 --workload triangles --scale 20
b bench_tri_s22 --workload triangles --scale 22
b bench_tri_s24 --workload triangles --scale 24
b bench_tri_s26 --workload triangles --scale 26 --steps 3 --warmup 1
b bench_c1 --workload c1
b bench_apply --workload apply
b bench_candidates --workload candidates
b bench_parse --workload parse
b bench_e2e_direct --workload e2e --staging direct --no-cpu-baseline
b e2e_c5_triangles_s23_1e8 --workload e2e --e2e-kind triangles --scale 23 --windows-edges 1e8 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_tri26 -o run --output-format csv -- python3 bench.py --workload triangles --scale 26 --steps 2 --warmup 1 --no-cpu-baseline > $O/trace_tri26.log 2>&1
echo all done
