#!/bin/bash
# round 4: float SUM presence inferred from a -0.0 identity -- bucket / parity / config-size float tests, then
# Double C2 against the previous build (variants/pre)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04fs
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bucket.py \
  tests/test_gpu_parity.py tests/test_gpu_chunked.py tests/test_gpu_stream.py \
  "tests/test_gpu_config_size.py::test_c2_full_window_double_within_tolerance" \
  "tests/test_gpu_config_size.py::test_c2_full_window_float_within_tolerance" > $O/tests.txt 2>&1
echo tests done
pre=$PWD/gelly-streaming_amd/variants/pre/libgellyhip.so
b() { local name=$1; shift; timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 "$@" > $O/$name.json 2> $O/$name.err; }
for i in 1 2 3; do
  b new_f64_$i --dtype float64; GELLY_HIP_LIB=$pre b pre_f64_$i --dtype float64
  echo "round $i done"
done
