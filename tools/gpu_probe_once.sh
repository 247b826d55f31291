# one-off GPU probe of round 5 (accumulate skew probe, HashSet simulation / emission A/B): bash tools/gpu_probe_once.sh TAG
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_candidates_chunked.py tests/test_gpu_config_size.py -k "cand or Cand or hashset or jdk or c5" > $O/tests.txt 2>&1
echo tests done
for v in base hub16; do
  if [ $v = base ]; then lib=gelly-streaming_amd/libgellyhip.so; else lib=gelly-streaming_amd/variants/$v/libgellyhip.so; fi
  GELLY_HIP_LIB=$lib timeout -k 10 200 python3 tools/accum_probe.py >> $O/probe_$v.txt 2>&1
  echo "$v done"
done
GS_HS_JDK_SERIAL=1 GS_CAND_SPLIT=0 timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline > $O/cand_r04kernels.json 2> $O/cand_r04kernels.err
echo r04 kernels done
timeout -k 10 300 python3 bench.py --workload cand_stream > $O/cand_new.json 2> $O/cand_new.err
echo new done
