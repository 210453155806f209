#!/bin/bash
# Runs scripts/pipe_order_probe.py for every STEP (two rank processes on the one GPU), then the slow case with rank
# 0 under rocprofv3 (kernel + HIP runtime trace) for the cause. Output under gpurun_out/pipeorder_TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/pipeorder_${1:-run}; rm -rf $O; mkdir -p $O
export NCCL_AMD_SPIN_TIMEOUT_MS=20000 MASTER_ADDR=127.0.0.1 WORLD_SIZE=2
pair() {  # STEP, prefix for rank 0 (e.g. a profiler command)
  export STEP=$1 MASTER_PORT=$((29500 + RANDOM % 1000)); shift
  RANK=1 LOCAL_RANK=1 timeout -k 10 200 python3 -u scripts/pipe_order_probe.py > $O/$STEP.r1.log 2>&1 &
  local p1=$!
  RANK=0 LOCAL_RANK=0 timeout -k 10 200 "$@" python3 -u scripts/pipe_order_probe.py > $O/$STEP.r0.log 2>&1
  local rc=$?
  wait $p1; local rc1=$?
  grep -h '^{' $O/$STEP.r0.log $O/$STEP.r1.log
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ]
}
if [ -n "$QUEUE_LIMITS" ]; then  # the box's queue scheduling parameters, then rank 0 alone with the extra queues
  for f in sched_policy hws_max_conc_proc mes cwsr_enable num_kcq compute_multipipe; do
    echo "amdgpu.$f=$(cat /sys/module/amdgpu/parameters/$f 2>/dev/null || echo n/a)"; done
  timeout -k 10 60 rocminfo 2>/dev/null | grep -iE "queue|Marketing|Compute Unit" | sort | uniq -c | head -20
  pair events_r0 || exit 1
  exit 0
fi
if [ -n "$QUEUE_VARIANTS" ]; then  # the same slow step under fewer / more hardware queues per process
  for q in 1 2 8; do echo "GPU_MAX_HW_QUEUES=$q"; GPU_MAX_HW_QUEUES=$q pair events || exit 1; done
  for s in events1 launch_other; do pair $s || exit 1; done
  exit 0
fi
for s in streams events copies pipe pipe_sync; do pair $s || exit 1; done
pair pipe rocprofv3 --kernel-trace --hip-runtime-trace -d $O/prof -o r0 --
