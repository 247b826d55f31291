#!/bin/bash
# round 4: light triangle chunks in phase order (parity + s24 / s26 A/B), C5 stream with the one-pass consumer
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP \
  tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_threads.py \
  "tests/test_gpu_config_size.py::test_c4_shape_triangles_vs_forward_algorithm" > $O/tests.txt 2>&1
echo tests done
for S in 24 26; do
  timeout -k 10 400 python3 bench.py --workload triangles --scale $S --steps 3 --warmup 1 --no-cpu-baseline > $O/tri_s${S}_lph.json 2> $O/tri_s${S}_lph.err
  echo tri s$S phased done
  GS_TH_LPHASED=0 timeout -k 10 400 python3 bench.py --workload triangles --scale $S --steps 3 --warmup 1 --no-cpu-baseline > $O/tri_s${S}_nolph.json 2> $O/tri_s${S}_nolph.err
  echo tri s$S unphased done
done
timeout -k 10 240 python3 bench.py --workload cand_stream > $O/cand_stream.json 2> $O/cand_stream.err
echo all done
