#!/bin/bash
# ReduceScatter / AllGather small-size sweep, LL protocol (default size table) vs SIMPLE (NCCL_PROTO=^LL),
# 2 ranks on the box's one GPU through the native driver (CU-masked streams, so no fork/join).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_SPIN_TIMEOUT_MS=20000 NCCL_AMD_FORK_JOIN=0
for c in rs ag; do
  timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c $c -b 64 -e 1048576 -f 4 -i 200 -w 20 > gpurun_out/native_${c}_ll.txt 2>&1 &&
  NCCL_PROTO=^LL timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c $c -b 64 -e 1048576 -f 4 -i 200 -w 20 > gpurun_out/native_${c}_simple.txt 2>&1 &&
  timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c $c -b 64 -e 262144 -f 4 -i 200 -w 20 -g 1 > gpurun_out/native_${c}_ll_graph.txt 2>&1 ||
  exit 1
done
for f in gpurun_out/native_{rs,ag}_*.txt; do echo "== $f"; cat $f; done
# Reduce (root 0): LL vs SIMPLE direct
timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c reduce -b 64 -e 1048576 -f 4 -i 200 -w 20 > gpurun_out/native_reduce_ll.txt 2>&1 &&
NCCL_PROTO=^LL timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c reduce -b 64 -e 1048576 -f 4 -i 200 -w 20 > gpurun_out/native_reduce_simple.txt 2>&1 &&
cat gpurun_out/native_reduce_ll.txt gpurun_out/native_reduce_simple.txt
