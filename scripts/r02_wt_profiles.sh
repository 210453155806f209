#!/bin/bash
# Round-2 call after the write-through copy store became the nRanks==1 default: the full GPU suite, the N=1
# bench line, then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (separate runs) of the same
# workload. Every GPU step bounded; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
O=gpurun_out/r02wt; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo bench failed; tail $O/bench_n1.err; exit 1; }
tail -c 1500 $O/bench_n1.json; echo
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1_trace -o run -- $B > $O/n1_trace.log 2>&1 || { echo n1 trace failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/n1_fetch -o run -- $B > $O/n1_fetch.log 2>&1 || { echo n1 fetch failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/n1_write -o run -- $B > $O/n1_write.log 2>&1 || { echo n1 write failed; exit 1; }
echo N1_PROFILES_OK
