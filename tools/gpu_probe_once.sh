# one-off GPU probe of round 5: candidate emission, the fast step's row state carried from the previous fast step
# (variants/carry) against the closed-form row search every step (variants/lane4)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
GELLY_HIP_LIB=gelly-streaming_amd/variants/carry/libgellyhip.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_candidates_chunked.py tests/test_gpu_api.py -k "cand or chunk or u32" > $O/tests_cand.log 2>&1
echo tests done
for rep in 1 2; do
  for v in lane4 carry; do
    for mode in "u32 none" "i64 none"; do
      set -- $mode
      GELLY_HIP_LIB=gelly-streaming_amd/variants/$v/libgellyhip.so timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline --cand-ids $1 --cand-consumer $2 > $O/${v}_${1}_${2}_$rep.json 2> $O/${v}_${1}_${2}_$rep.err
    done
    echo $v $rep done
  done
done
echo done
