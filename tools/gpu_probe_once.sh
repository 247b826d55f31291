# round-5 final evidence, part 1: the whole -m gpu suite, smoke(), the default bench line, the forced exchange
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests_full_suite.txt 2>&1
echo tests done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
echo smoke done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
echo bench done
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 timeout -k 10 300 python3 bench.py --force-exchange --no-cpu-baseline > $O/forced.json 2> $O/forced.err
echo forced done
