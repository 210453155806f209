#!/bin/bash
# Round-2 measurement call: N=1 bench line + rocprofv3 kernel trace + PMC passes (separate runs), and the
# n=2 one-GPU channel sweep (256/128/64/32) under a kernel trace and FETCH/WRITE passes (rank 0 profiled,
# rank 1 a plain process). Every GPU step bounded; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
O=gpurun_out/r02p; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { echo bench failed; exit 1; }
tail -c 600 $O/bench_n1.json; echo
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1_trace -o run -- $B > $O/n1_trace.log 2>&1 || { echo n1 trace failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/n1_fetch -o run -- $B > $O/n1_fetch.log 2>&1 || { echo n1 fetch failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/n1_write -o run -- $B > $O/n1_write.log 2>&1 || { echo n1 write failed; exit 1; }
echo N1_PROFILES_OK
CFG=scripts/cfg/n2_channels.json
run2() {  # name, rocprof args...
  local name=$1; shift
  mkdir -p $O/$name
  timeout -k 10 200 python3 scripts/rank_sweep.py 1 2 $O/$name $CFG > $O/$name/r1.log 2>&1 &
  local P1=$!
  timeout -s KILL 200 rocprofv3 "$@" --output-format csv -d $O/$name/prof -o run -- python3 scripts/rank_sweep.py 0 2 $O/$name $CFG > $O/$name/r0.log 2>&1
  local R0=$?
  wait $P1; local R1=$?
  echo "$name rank0=$R0 rank1=$R1"
  [ $R0 -eq 0 ] && [ $R1 -eq 0 ]
}
run2 n2_trace --kernel-trace --stats && run2 n2_fetch --pmc FETCH_SIZE && run2 n2_write --pmc WRITE_SIZE && echo N2_PROFILES_OK
