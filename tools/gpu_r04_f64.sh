#!/bin/bash
# round 4: Double C2 -- kernel trace + FETCH / WRITE passes (write amplification of the unpacked partition)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O/pmc
timeout -k 10 300 python3 bench.py --dtype float64 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  -- python3 bench.py --dtype float64 --no-cpu-baseline --steps 5 > $O/trace.log 2>&1
for c in FETCH_SIZE:fetch WRITE_SIZE:write; do
  timeout -s KILL 150 rocprofv3 --pmc ${c%%:*} -d $O/pmc/${c#*:} -o run --output-format csv \
    -- python3 bench.py --dtype float64 --no-cpu-baseline --steps 3 --warmup 2 > $O/pmc_${c#*:}.log 2>&1
  echo "pmc ${c%%:*} done"
done
