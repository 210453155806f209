#!/bin/bash
# Round 3 N=1 evidence on the final build: rocprofv3 --kernel-trace --stats of the bench's own command, then the
# FETCH_SIZE and WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md §HBM), each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r03prof; rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1_trace -o run -- $B > $O/n1_trace.log 2>&1 || { echo trace failed; tail $O/n1_trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/n1_fetch -o run -- $B > $O/n1_fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/n1_write -o run -- $B > $O/n1_write.log 2>&1 || { echo write failed; exit 1; }
grep -h '^{' $O/n1_trace.log | tail -1
echo N1_PROFILES_OK
