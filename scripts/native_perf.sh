#!/bin/bash
# nccl-tests-style native driver (tests/native/nccl_perf, C ABI only) with 2 ranks on the box's one GPU.
# Its streams are CU-masked (a hardware queue each), so NCCL_AMD_FORK_JOIN=0 is safe for the timed runs;
# one run keeps the default fork/join (what plain streams need) for coverage.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_SPIN_TIMEOUT_MS=20000
NCCL_AMD_FORK_JOIN=0 timeout -k 10 200 ./tests/native/nccl_perf -r 2 -b 8 -e 268435456 -f 4 -i 20 > gpurun_out/native_eager.txt 2>&1 && echo EAGER_OK &&
NCCL_AMD_FORK_JOIN=0 timeout -k 10 200 ./tests/native/nccl_perf -r 2 -b 8 -e 4194304 -f 4 -i 50 -g 1 > gpurun_out/native_graph.txt 2>&1 && echo GRAPH_OK &&
NCCL_AMD_FORK_JOIN=0 timeout -k 10 200 ./tests/native/nccl_perf -r 2 -b 8 -e 16777216 -f 8 -i 20 -t bf16 -o max > gpurun_out/native_bf16_max.txt 2>&1 && echo BF16_OK &&
timeout -k 10 200 ./tests/native/nccl_perf -r 2 -b 1024 -e 1048576 -f 32 -i 10 -g 1 > gpurun_out/native_forkjoin_graph.txt 2>&1 && echo FJ_OK
