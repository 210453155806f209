#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
for f in ${FLAGS:-0 1 2 4 7}; do
  NCCL_AMD_PROTO_FLAGS=$f timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600+f)) bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_n2_f$f.log 2>&1
  echo "flags=$f rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_n2_f$f.log) $(grep -o 'CHECK FAILED.*mismatches' gpurun_out/bench_n2_f$f.log | head -1)"
done
