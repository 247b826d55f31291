#!/bin/bash
# round 4: k_bk_accum's packed records as one stream per item (the speculative partition's segment
# pieces no longer drain the loads in flight) -- bucket / parity tests, then A/B against the previous
# build (variants/pre) on C2 (packed Long SUM) and the C3 fold, same box
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04flat}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bucket.py \
  tests/test_gpu_parity.py tests/test_gpu_chunked.py tests/test_gpu_config_size.py > $O/tests.txt 2>&1
echo tests done
pre=$PWD/gelly-streaming_amd/variants/pre/libgellyhip.so
b() { local name=$1; shift; timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err; }
for i in 1 2 3; do
  b new_c2_$i; GELLY_HIP_LIB=$pre b pre_c2_$i
  echo "round $i done"
done
b new_c3 --workload fold; GELLY_HIP_LIB=$pre b pre_c3 --workload fold
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_new -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace_new.log 2>&1
echo trace done
