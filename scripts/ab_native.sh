#!/bin/bash
# A/B of the previous library (ablib/libnccl.so.2, picked up through LD_LIBRARY_PATH ahead of the driver's
# RUNPATH) against the current one: small-size graph-replayed AllReduce latency, alternating runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_SPIN_TIMEOUT_MS=10000 NCCL_AMD_FORK_JOIN=0
for i in 1 2 3; do
  for L in prev cur; do
    if [ $L = prev ]; then LP=$PWD/ablib; else LP=""; fi
    for R in ${RANKS:-2 4}; do
      LD_LIBRARY_PATH=$LP timeout -k 10 60 ./tests/native/nccl_perf -r $R -b 8 -e 65536 -f 8 -i 200 -w 20 -g 1 ${AB_ARGS} \
        > gpurun_out/abn.txt 2>&1 || { echo "run failed"; cat gpurun_out/abn.txt; exit 1; }
      echo "$L r=$R $(grep -v '^#' gpurun_out/abn.txt | awk '{printf "%s:%s ", $1, $3}')"
    done
  done
done
