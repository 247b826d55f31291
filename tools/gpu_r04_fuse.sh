#!/bin/bash
# round 4 A/B: the unique oriented edges straight into out-lists (GS_TRI_FUSED_UNIQUE 1, default) vs
# reduce-by-key + k_tri_out (0) -- every triangle test, then s24 / s26 bench lines, same box
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r04fuse}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_tri_degree_sample.py \
  tests/test_gpu_tri_variants.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_threads.py \
  tests/test_gpu_stream.py "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" \
  "tests/test_gpu_config_size.py::test_c4_window_s26_triangles_vs_forward_algorithm" > $O/tests.txt 2>&1
echo tests done
b() { local name=$1 k=$2; shift 2; GS_TRI_FUSED_UNIQUE=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload triangles "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b s24_fu_1 1 --scale 24
b s24_rbk_1 0 --scale 24
b s24_fu_2 1 --scale 24
b s24_rbk_2 0 --scale 24
b s26_fu 1 --scale 26 --steps 3 --warmup 1
b s26_rbk 0 --scale 26 --steps 3 --warmup 1
