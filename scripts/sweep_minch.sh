#!/bin/bash
# direct-path channel granularity sweep (NCCL_AMD_MIN_CHANNEL_BYTES) with the N=2 one-GPU rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
i=0
for M in 32768 65536 131072 262144; do
  i=$((i+1))
  NCCL_AMD_MIN_CHANNEL_BYTES=$M timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29850 + i)) bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/minch_$M.log 2>&1 || { echo "run $M failed"; exit 1; }
  echo "run $M ok"
done
