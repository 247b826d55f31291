# one-off GPU probe of round 5: C5 consumer in turn vs overlapped, chunk sizes
set -e
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 300 python3 bench.py --workload cand_stream --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err; echo "$name done"; }
b serial_c28
b overlap_c28 --cand-overlap
b serial_c26 --chunk-records 67108864
b serial_c25 --chunk-records 33554432
b serial_c24 --chunk-records 16777216
