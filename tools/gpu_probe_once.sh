# one-off GPU probe of round 5: 9-bit-digit triangle sorts (parity + same-box A/B)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_tri_variants.py tests/test_gpu_config_size.py tests/test_gpu_tri_degree_sample.py -k "tri or c4" > $O/tests.txt 2>&1
echo tests done
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/d9_$rep.json 2> $O/d9_$rep.err
  echo d9 $rep done
  GS_SORT_DIGIT9=0 timeout -k 10 300 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/d8_$rep.json 2> $O/d8_$rep.err
  echo d8 $rep done
done
