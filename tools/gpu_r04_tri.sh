#!/bin/bash
# round 4: oriented-key unroll (GS_TRI_OKEYS_UNROLL / _SPLIT) parity + A/B at s26, sort tile-shape variants
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fresh_process.py tests/test_gpu_tri_variants.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" > $O/tests.txt 2>&1
echo tests done
A="--workload triangles --scale 26 --steps 2 --warmup 1 --no-cpu-baseline"
tb() { local name=$1; shift; env "$@" timeout -k 10 300 python3 bench.py $A > $O/$name.json 2> $O/$name.err; echo "$name done"; }
tb u4_split GS_TRI_OKEYS_UNROLL=4
tb u1_split GS_TRI_OKEYS_UNROLL=1
tb u4_nosplit GS_TRI_OKEYS_UNROLL=4 GS_TRI_OKEYS_SPLIT=0
tb u2_split GS_TRI_OKEYS_UNROLL=2
tb u4_split_x1 GS_TH_XCD=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $A > $O/trace.log 2>&1
echo trace done
for v in sb256i16 sb512i8 sb1024i8; do
  tb var_$v GELLY_HIP_LIB=$PWD/gelly-streaming_amd/variants/$v/libgellyhip.so
done
echo all done
