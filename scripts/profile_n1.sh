#!/bin/bash
# rocprofv3 kernel-trace + PMC passes (separate runs) for the N=1 bench workload (256 MiB fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- $B > gpurun_out/prof/trace.log 2>&1 && echo TRACE_OK &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- $B > gpurun_out/prof/fetch.log 2>&1 && echo FETCH_OK &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- $B > gpurun_out/prof/write.log 2>&1 && echo WRITE_OK
