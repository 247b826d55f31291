# one-off GPU probe of round 5: light count with contiguous queue ranges per wave (A/B, s24 + s26)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
GELLY_HIP_LIB=gelly-streaming_amd/variants/lblk/libgellyhip.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tri_variants.py tests/test_gpu_config_size.py -k "tri and not s26" > $O/tests.txt 2>&1
echo tests done
for rep in 1 2; do
  for v in base lblk; do
    if [ "$v" = base ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --workload triangles --scale 26 --steps 3 --warmup 1 --no-cpu-baseline > $O/s26_${v}_$rep.json 2> $O/s26_${v}_$rep.err
    GELLY_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --workload triangles --scale 24 --no-cpu-baseline > $O/s24_${v}_$rep.json 2> $O/s24_${v}_$rep.err
    echo $v $rep done
  done
done
