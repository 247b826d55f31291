#!/bin/bash
# Round-2 evidence for the C2 headline: the default bench line (with CPU baseline), a rocprofv3
# kernel-trace summary of the same command, and FETCH_SIZE / WRITE_SIZE passes (separate runs)
# for profiles/pmc_traffic.json.  Run on the GPU box from the repo root:  bash tools/profile_c2.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r02}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench_c2_i64.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  d=$O/pmc/$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 150 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/pmc_$c.log 2>&1
done
python3 tools/pmc_traffic.py $O/pmc -o $O/pmc_traffic.json
