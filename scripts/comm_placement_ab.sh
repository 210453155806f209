#!/bin/bash
# Identical-plan communicators timed side by side (n = 2 ranks, one GPU): the staged tuning part alone with the default
# column repeated (BENCH_TUNING_COLS), REPS interleaved rounds; does a communicator's own staging slab make it faster or
# slower than an identical one? Two launches, so per-launch placement shows too. Output gpurun_out/placement_*.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000 BENCH_SUITE_PARTS=staged_tuning BENCH_TUNING_COLS=${COLS:-0,0,0,0,0,0} BENCH_TUNING_REPS=${REPS:-5}
for L in 1 2; do
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29700 + L)) bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-extra \
    > gpurun_out/placement_$L.log 2>&1 || { echo "launch $L failed"; exit 1; }
  grep '^{' gpurun_out/placement_$L.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('launch $L headline ms', d['ms_per_step'])
for r in d['suite']['staged_tuning']['runs']: print('  ', r['env'], r['ms'], r['ms_min'], r['ms_max'])"
done
