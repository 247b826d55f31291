# one-off GPU probe of round 5: accumulate item order (LPT) A/B + bucket tests
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bucket.py > $O/tests.txt 2>&1
echo tests done
for rep in 1 2; do
  for v in base pre; do
    if [ "$v" = base ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err
    echo $v $rep done
  done
done
