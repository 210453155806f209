#!/bin/bash
# Multi-rank rehearsal on the one-GPU box: every rank is its own process on the same GPU (IPC path).
# Exercises bench.py's N>1 code (uid exchange, barriers, max-over-ranks, suite) — not xGMI.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
for NP in ${NPS:-2 4}; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
    --master-port $((29600 + NP)) bench.py --gpus $NP --steps 10 --warmup 3 --cpu-seconds 2 ${REH_ARGS:---quick-suite} \
    > gpurun_out/rehearse_n$NP.log 2>&1 || { echo "N=$NP FAILED rc=$?"; exit 1; }
  echo "N=$NP OK"
done
