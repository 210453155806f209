#!/bin/bash
# A/B of two libnccl.so builds on small-message latency: nccl_perf fp16 AllReduce 8 B .. 256 KiB, two ranks on one
# GPU (per-rank queues), A = abprev/ (make lib BUILD=build_ab LIBDIR=abprev from the base commit), B = this tree;
# ROUNDS interleaved rounds (default 3); AB_MAX = largest size (default 256 KiB), AB_TAG = output name (default ll);
# any NCCL_* setting in the environment applies to both. Output: gpurun_out/ab_<tag>_{A,B}_<round>.txt
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
for r in $(seq 1 "${ROUNDS:-3}"); do
  LD_LIBRARY_PATH=$PWD/abprev timeout -k 10 120 tests/native/nccl_perf -d 1 -r ${AB_RANKS:-2} ${AB_COLL:+-c $AB_COLL} -b 8 -e ${AB_MAX:-262144} -f 4 -t half -i 200 -w 20 -H 1 \
    > gpurun_out/ab_${AB_TAG:-ll}_A_$r.txt 2>&1
  timeout -k 10 120 tests/native/nccl_perf -d 1 -r ${AB_RANKS:-2} ${AB_COLL:+-c $AB_COLL} -b 8 -e ${AB_MAX:-262144} -f 4 -t half -i 200 -w 20 -H 1 > gpurun_out/ab_${AB_TAG:-ll}_B_$r.txt 2>&1
  echo "round $r ok"
done
