# one-off GPU probe of round 5: output buffers reused across windows vs allocated per window (same box)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/reuse_$rep.json 2> $O/reuse_$rep.err
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --alloc-outputs > $O/alloc_$rep.json 2> $O/alloc_$rep.err
  echo rep $rep done
done
