# one-off GPU probe of round 5: grid-stride merges (bucket tests + C2 / C3 lines, A/B against HEAD)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_chunked.py tests/test_gpu_config_size.py -k "not s26" > $O/tests.txt 2>&1
echo tests done
for rep in 1 2; do
  for v in base pre; do
    if [ "$v" = base ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --workload fold --stream zipf --no-cpu-baseline > $O/zipf_${v}_$rep.json 2> $O/zipf_${v}_$rep.err
    echo $v $rep done
  done
done
