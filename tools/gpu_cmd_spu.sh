set -e
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_config_size.py tests/test_gpu_dist.py tests/test_gpu_chunked.py tests/test_gpu_api.py -k "not s26 and not c5" > gpurun_out/t_spu.txt 2>&1 || { tail -30 gpurun_out/t_spu.txt; exit 1; }
tail -1 gpurun_out/t_spu.txt
mkdir -p gpurun_out/spu
for w in "c3_rmat --workload fold" "c3_zipf --workload fold --stream zipf" "c2_f64 --dtype float64" "tri_s24 --workload triangles --scale 24 --steps 3 --warmup 1" "c2 "; do
  set -- $w; name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > gpurun_out/spu/$name.json 2>/dev/null
  echo "$name done"
done
