#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
i=0
run() { # label, env...
  local label=$1; shift; i=$((i+1))
  env "$@" timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700+i)) bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline ${SIZE:+--size-mib $SIZE} > gpurun_out/bis_$label.log 2>&1
  echo "$label rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bis_$label.log) $(grep -o 'CHECK FAILED.*mismatches of [0-9]*' gpurun_out/bis_$label.log | head -1)"
}
run old NCCL_AMD_LIB=$PWD/oldlib/libnccl_2bc8a99.so
#run old_b NCCL_AMD_LIB=$PWD/oldlib/libnccl_2bc8a99.so
#run new_ch1 NCCL_MAX_CTAS=1
run new_ch8 NCCL_MAX_CTAS=8
run new_ch32 NCCL_MAX_CTAS=32
run new_slots1 NCCL_AMD_NSLOTS=1
#run new_slots4 NCCL_AMD_NSLOTS=4
SIZE=16 run new_16m
run new_elementwise NCCL_AMD_FORCE_ELEMENTWISE=1
