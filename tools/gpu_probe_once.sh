# one-off GPU probe of round 5: the dist line's reused outputs (forced exchange, world 1) + fold line
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --force-exchange --no-cpu-baseline > $O/forced_reuse_$rep.json 2> $O/forced_reuse_$rep.err
  timeout -k 10 300 python3 bench.py --force-exchange --no-cpu-baseline --alloc-outputs > $O/forced_alloc_$rep.json 2> $O/forced_alloc_$rep.err
  echo rep $rep done
done
unset WORLD_SIZE RANK LOCAL_RANK MASTER_ADDR MASTER_PORT
timeout -k 10 300 python3 bench.py --workload fold --no-cpu-baseline > $O/fold_reuse.json 2> $O/fold_reuse.err
timeout -k 10 300 python3 bench.py --workload fold --no-cpu-baseline --alloc-outputs > $O/fold_alloc.json 2> $O/fold_alloc.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2_reuse.json 2> $O/c2_reuse.err
echo done
