#!/bin/bash
# n = 8 one-GPU rehearsal of the headline alone (no suite), every rank logging at TRACE level into gpurun_out/reh8/,
# repeated RUNS times (stops at the first failed check): the eager path with bounced ranks under a full trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
rm -rf gpurun_out/reh8; mkdir -p gpurun_out/reh8
for RUN in $(seq 1 ${RUNS:-2}); do
  mkdir -p gpurun_out/reh8/run$RUN
  NCCL_DEBUG=TRACE NCCL_DEBUG_FILE=$PWD/gpurun_out/reh8/run$RUN/%p.log timeout -k 10 200 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29750 + RUN)) bench.py --gpus 8 --steps 10 \
    --warmup 3 --no-cpu-baseline --no-extra --no-suite > gpurun_out/reh8/run$RUN/bench.log 2>&1 || { echo "run $RUN rc=$?"; exit 1; }
  grep -o "\"check\": \"[a-zA-Z]*\"" gpurun_out/reh8/run$RUN/bench.log | head -1
  grep -q '"check": "FAIL"' gpurun_out/reh8/run$RUN/bench.log && { echo "run $RUN: check FAIL"; exit 0; }
  echo "run $RUN ok"
done
