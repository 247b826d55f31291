# one-off GPU probe of round 5: C5 with uint32 id columns, consumer variants
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline --cand-ids u32 > $O/c5_u32_sum.json 2> $O/c5_u32_sum.err
timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline --cand-ids u32 --cand-overlap > $O/c5_u32_sum_overlap.json 2> $O/c5_u32_sum_overlap.err
timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline --cand-ids u32 --chunk-records 134217728 > $O/c5_u32_sum_c27.json 2> $O/c5_u32_sum_c27.err
timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline --cand-ids u32 --chunk-records 536870912 > $O/c5_u32_sum_c29.json 2> $O/c5_u32_sum_c29.err
echo done
