#!/bin/bash
# Round-2 first GPU call: n=2 two-process rehearsal sweep (plain, then rank 0 under rocprofv3 kernel trace),
# then the IPC-stall diagnostic. Every GPU step is time-bounded; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
O=gpurun_out/r02c1; rm -rf $O; mkdir -p $O/plain $O/traced
CFG=${CFG:-scripts/cfg/n2_sweep.json}
timeout -k 10 240 python3 scripts/rank_sweep.py 1 2 $O/plain $CFG > $O/plain/r1.log 2>&1 &
P1=$!
timeout -k 10 240 python3 scripts/rank_sweep.py 0 2 $O/plain $CFG > $O/plain/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "plain sweep rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || exit 1
timeout -k 10 240 python3 scripts/rank_sweep.py 1 2 $O/traced $CFG > $O/traced/r1.log 2>&1 &
P1=$!
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/traced/prof -o run -- \
  python3 scripts/rank_sweep.py 0 2 $O/traced $CFG > $O/traced/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "traced sweep rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || exit 1
[ "${SKIP_DIAG:-0}" = 1 ] && exit 0
timeout -k 10 200 python3 scripts/ipc_hang_diag.py $O/diag 4 524288 > $O/diag.log 2>&1; echo "diag rc=$?"
tail -3 $O/diag.log
