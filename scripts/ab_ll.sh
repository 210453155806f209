#!/bin/bash
# A/B of two libnccl.so builds on the same box: N=2 rehearsal sweeps (quick suite), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
i=0
for L in ablib/libnccl_prev.so nccl_amd/lib/libnccl.so ablib/libnccl_prev.so nccl_amd/lib/libnccl.so; do
  i=$((i+1))
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29800 + i)) bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --quick-suite > gpurun_out/ab_$i.log 2>&1 || { echo "run $i failed"; exit 1; }
  echo "run $i ($L) ok"
done
