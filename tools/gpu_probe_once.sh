# round-5 final evidence, part 2: the secondary bench lines DESIGN.md quotes
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b bench_c2_f64 --dtype float64
b bench_c3_rmat --workload fold
b bench_c3_zipf --workload fold --stream zipf
b bench_tri_s24 --workload triangles --scale 24
b bench_tri_s26 --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline
b bench_cc_s24 --workload cc
b bench_cand_stream --workload cand_stream --no-cpu-baseline
