#!/bin/bash
# Round 3: roctx ranges on the API entry points (NCCL_AMD_ROCTX=1): rocprofv3 --marker-trace (+ kernel trace) of a
# 2-rank AllReduce (both ranks in one process, 5 timed steps + 3 warm-up, one ncclGroupStart/End per step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r03roctx
mkdir -p $D
NCCL_AMD_ROCTX=1 STEPS=5 MODE=direct timeout -k 10 200 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
  -d $D -o run -- python3 scripts/multirank_one_gpu.py > $D/run.log 2>&1 || { echo "roctx trace failed"; tail -5 $D/run.log; exit 1; }
echo "roctx ok"; ls $D
