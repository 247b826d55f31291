#!/bin/bash
# round 4: vectorized loads of the unpacked partition in k_bk_accum -- bucket / parity tests, then A/B
# against the previous build (variants/pre) on Double C2, C3 fold (R-MAT / Zipf) and the packed C2
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bucket.py \
  tests/test_gpu_parity.py tests/test_gpu_chunked.py "tests/test_gpu_config_size.py::test_c2_full_window_double_within_tolerance" \
  "tests/test_gpu_config_size.py::test_c3_full_window_degree_max" "tests/test_gpu_config_size.py::test_c2_full_window_float_within_tolerance" \
  > $O/tests.txt 2>&1
echo tests done
pre=$PWD/gelly-streaming_amd/variants/pre/libgellyhip.so
b() { local name=$1; shift; timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 "$@" > $O/$name.json 2> $O/$name.err; }
for i in 1 2; do
  b new_f64_$i --dtype float64; GELLY_HIP_LIB=$pre b pre_f64_$i --dtype float64
  b new_c3_$i --workload fold; GELLY_HIP_LIB=$pre b pre_c3_$i --workload fold
  b new_zipf_$i --workload fold --stream zipf; GELLY_HIP_LIB=$pre b pre_zipf_$i --workload fold --stream zipf
  b new_c2_$i; GELLY_HIP_LIB=$pre b pre_c2_$i
  echo "round $i done"
done
