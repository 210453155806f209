#!/bin/bash
# n = 8 one-GPU rehearsal of the staged tuning part alone, with per-part tracing (a stalled column shows in the log),
# without the harness line-up before each warm-up (BENCH_NO_LINEUP=1): the co-residency cap alone must prevent stalls
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000 BENCH_TRACE=1 BENCH_SUITE_PARTS=staged_tuning BENCH_NO_LINEUP=1
NP=${NP:-8}
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
  --master-port 29711 bench.py --gpus $NP --steps 10 --warmup 3 --no-cpu-baseline --no-extra \
  > gpurun_out/reh_tuning_n$NP.log 2>&1 || { echo "N=$NP FAILED rc=$?"; exit 1; }
echo "N=$NP OK"
