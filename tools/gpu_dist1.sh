#!/bin/bash
# The multi-GPU code path at world size 1 on one box: torchrun with the ABI's own RCCL exchange
# (gs_window_reduce_dist, GS_FLAG_TEST_FORCE_EXCHANGE off: world 1 skips the exchange) and the torch one,
# against the plain single-GPU step.  bash tools/gpu_dist1.sh TAG
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dist1}
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline > "$O/single.json" 2> "$O/single.err"
for ex in abi torch; do
  for w in reduce fold triangles; do
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --steps 10 --workload $w --exchange $ex --no-cpu-baseline \
      > "$O/torchrun_${ex}_$w.json" 2> "$O/torchrun_${ex}_$w.err"
    echo "$ex $w done"
  done
done
# the exchange's own cost at world 1: owner partition + RCCL self-exchange + merge on every window
for w in reduce fold; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 1 --steps 10 --workload $w --exchange abi --force-exchange --no-cpu-baseline \
    > "$O/torchrun_abi_forced_$w.json" 2> "$O/torchrun_abi_forced_$w.err"
  echo "forced $w done"
done
