# one-off GPU probe of round 5: the keyBy exchange at world size 1 (forced), bench lines + kernel trace
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm_group.py tests/test_gpu_dist.py > $O/tests.txt 2>&1
echo tests done
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
timeout -k 10 300 python3 bench.py --force-exchange --no-cpu-baseline > $O/forced.json 2> $O/forced.err
echo forced done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/plain.json 2> $O/plain.err
echo plain done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --force-exchange --no-cpu-baseline --steps 20 --warmup 5 > $O/trace.log 2>&1
echo trace done
