# one-off GPU probe of round 5: candidates parity, then C5 emission A/B: bash tools/gpu_probe_once.sh TAG
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_dist.py tests/test_gpu_candidates_chunked.py tests/test_gpu_config_size.py -k "cand or Cand or hashset or jdk or c5" > $O/tests.txt 2>&1
echo tests done
for rep in 1 2; do
timeout -k 10 300 python3 bench.py --workload cand_stream --cand-windows 1 --cand-consumer none --no-cpu-baseline > $O/split_$rep.json 2>$O/split_$rep.err
GS_CAND_SPLIT=0 timeout -k 10 300 python3 bench.py --workload cand_stream --cand-windows 1 --cand-consumer none --no-cpu-baseline > $O/nosplit_$rep.json 2>$O/nosplit_$rep.err
echo rep $rep done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload cand_stream --cand-windows 1 --max-chunks 40 --cand-consumer none --no-cpu-baseline > $O/trace.log 2>&1
echo trace done
