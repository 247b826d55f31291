#!/bin/bash
# round 4: the C2 headline (bench + kernel trace + PMC traffic) and the candidate emission's trace / PMC
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
bash tools/gpu.sh c2 r04p
echo c2 done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d "$PWD/$O/pmc_cand_$c" -o run --output-format csv \
    -- python3 bench.py --workload cand_stream --max-chunks 6 > $O/pmc_cand_$c.log 2>&1
  echo pmc $c done
done
timeout -k 10 400 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 > $O/tri_s26.json 2> $O/tri_s26.err
echo tri s26 done
timeout -k 10 300 python3 bench.py --workload fold > $O/c3_rmat.json 2> $O/c3_rmat.err
timeout -k 10 300 python3 bench.py --dtype float64 > $O/c2_f64.json 2> $O/c2_f64.err
echo all done
