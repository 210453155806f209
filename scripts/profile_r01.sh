#!/bin/bash
# rocprofv3 kernel-trace + PMC passes for the N=1 bench workload, and a 2-rank bench rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- $B > gpurun_out/prof/trace.log 2>&1 && echo TRACE_OK &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- $B > gpurun_out/prof/fetch.log 2>&1 && echo FETCH_OK &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- $B > gpurun_out/prof/write.log 2>&1 && echo WRITE_OK &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_n2_onegpu.log 2>&1 && echo BENCH2_OK
