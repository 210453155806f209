# shared helper for the one-GPU multi-rank sweeps (sourced)
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
i=0
run() {  # $1 = label, rest = env assignments
  local label=$1; shift; i=$((i+1))
  env "$@" timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} \
    --master-addr 127.0.0.1 --master-port $((29500 + i)) bench.py --gpus ${NP:-2} --steps ${STEPS:-20} --warmup 5 \
    --no-cpu-baseline ${SIZE:+--size-mib $SIZE} > gpurun_out/tune_$label.log 2>&1
  echo "$label rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune_$label.log) $(grep -o '"check": "[a-zA-Z]*"' gpurun_out/tune_$label.log)"
}
