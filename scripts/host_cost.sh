#!/bin/bash
# Host issue cost vs device time of small collectives (native driver, hold mode: the streams are held by a
# spin kernel while the timed collectives are issued). 1 rank (copy kernel) and 2 ranks on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_SPIN_TIMEOUT_MS=20000 NCCL_AMD_FORK_JOIN=0
timeout -k 10 60 ./scripts/launch_probe > gpurun_out/launch_probe.txt 2>&1 &&
timeout -k 10 120 ./tests/native/nccl_perf -r 1 -b 8 -e 262144 -f 8 -i 100 -w 50 -H 1 > gpurun_out/host_r1.txt 2>&1 &&
timeout -k 10 120 ./tests/native/nccl_perf -r 2 -b 8 -e 262144 -f 8 -i 100 -w 50 -H 1 > gpurun_out/host_r2.txt 2>&1 &&
timeout -k 10 120 ./tests/native/nccl_perf -r 2 -c rs -b 64 -e 262144 -f 8 -i 100 -w 50 -H 1 > gpurun_out/host_r2_rs.txt 2>&1 &&
timeout -k 10 120 ./tests/native/nccl_perf -r 2 -b 8 -e 262144 -f 8 -i 500 -w 50 > gpurun_out/host_r2_eager.txt 2>&1
cat gpurun_out/launch_probe.txt gpurun_out/host_r1.txt gpurun_out/host_r2.txt gpurun_out/host_r2_rs.txt gpurun_out/host_r2_eager.txt
