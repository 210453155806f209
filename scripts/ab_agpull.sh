#!/bin/bash
# Staged path push vs pull variants (NCCL_AMD_AG_PULL / NCCL_AMD_RS_PULL): multi-process parity, then
# one-GPU timings through the native driver (HBM-bound here; the 8-GPU suite measures xGMI).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=10000 NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_collectives.py -v --timeout 300 --timeout-method thread -k "multi_process" > gpurun_out/agpull.log 2>&1; grep -E "PASS|FAIL" gpurun_out/agpull.log | tail -14
timeout -k 10 100 ./tests/native/nccl_perf -r 2 -b 1048576 -e 268435456 -f 16 -i 20 > gpurun_out/push.txt 2>&1 && NCCL_AMD_AG_PULL=1 timeout -k 10 100 ./tests/native/nccl_perf -r 2 -b 1048576 -e 268435456 -f 16 -i 20 > gpurun_out/pull.txt 2>&1 && NCCL_AMD_RS_PULL=1 NCCL_AMD_AG_PULL=1 timeout -k 10 100 ./tests/native/nccl_perf -r 2 -b 1048576 -e 268435456 -f 16 -i 20 > gpurun_out/pull2.txt 2>&1 && NCCL_AMD_RS_PULL=1 timeout -k 10 100 ./tests/native/nccl_perf -r 2 -c rs -b 1048576 -e 268435456 -f 16 -i 20 > gpurun_out/pull3.txt 2>&1; cat gpurun_out/push.txt gpurun_out/pull.txt gpurun_out/pull2.txt gpurun_out/pull3.txt
