#!/bin/bash
# Round 2, pass q: new tests (treeified flag, components, split triangles) + the bench lines of every workload
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r2q
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_components.py -v -m gpu -k "treeified or components or tri" --timeout 200 --timeout-method thread > gpurun_out/r2q/tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
B="timeout -k 10 300 python bench.py"
$B > gpurun_out/r2q/c2_i64.json 2> gpurun_out/r2q/c2_i64.err || exit 1
$B --dtype float64 > gpurun_out/r2q/c2_f64.json 2> gpurun_out/r2q/c2_f64.err || exit 1
$B --workload fold > gpurun_out/r2q/c3_rmat.json 2> gpurun_out/r2q/c3_rmat.err || exit 1
$B --workload fold --stream zipf > gpurun_out/r2q/c3_zipf.json 2> gpurun_out/r2q/c3_zipf.err || exit 1
$B --workload cc --steps 5 --warmup 2 > gpurun_out/r2q/cc_s24.json 2> gpurun_out/r2q/cc_s24.err || exit 1
$B --workload triangles --scale 24 --steps 4 --warmup 1 > gpurun_out/r2q/tri_s24.json 2> gpurun_out/r2q/tri_s24.err || exit 1
