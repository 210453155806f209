#!/bin/bash
# Parity tests, then a parameter sweep of the multi-rank kernel with all ranks on the box's one GPU
# (protocol/HBM efficiency proxy; xGMI is not exercised here).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 600 python -m pytest tests -m gpu -x -v -s > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK || exit 1; fi
i=0
run() {  # $1 = label, rest = env assignments
  local label=$1; shift; i=$((i+1))
  env "$@" timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} \
    --master-addr 127.0.0.1 --master-port $((29500 + i)) bench.py --gpus ${NP:-2} --steps 20 --warmup 5 \
    --no-cpu-baseline > gpurun_out/tune_$label.log 2>&1
  echo "$label rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune_$label.log) $(grep -o '"check": "[a-zA-Z]*"' gpurun_out/tune_$label.log)"
}
run ch64 NCCL_MAX_CTAS=64
run ch128 NCCL_MAX_CTAS=128
run ch128_s64k NCCL_MAX_CTAS=128 NCCL_AMD_SLOT_BYTES=65536
run ch128_s256k NCCL_MAX_CTAS=128 NCCL_AMD_SLOT_BYTES=262144
run ch128_n3 NCCL_MAX_CTAS=128 NCCL_AMD_NSLOTS=3
run ch256_s64k NCCL_MAX_CTAS=256 NCCL_AMD_SLOT_BYTES=65536
