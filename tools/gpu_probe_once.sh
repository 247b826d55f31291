# one-off GPU probe of round 5: owner-grouped emit for the keyBy exchange (tests + forced-exchange line + trace)
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_comm_group.py tests/test_gpu_dist.py -k "reduce or fold or rccl or merges or miss" > $O/tests.txt 2>&1
echo tests done
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --force-exchange --no-cpu-baseline > $O/forced_$rep.json 2> $O/forced_$rep.err
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/plain_$rep.json 2> $O/plain_$rep.err
  echo rep $rep done
done
timeout -k 10 300 python3 bench.py --force-exchange --workload fold --no-cpu-baseline > $O/forced_fold.json 2> $O/forced_fold.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --force-exchange --no-cpu-baseline --steps 20 --warmup 5 > $O/trace.log 2>&1
echo trace done
