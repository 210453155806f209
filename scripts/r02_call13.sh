#!/bin/bash
# Round 2 call 13: full-size BASELINE-config parity, N=1 bench line, n=2 sweep regression check after the
# collKernel refactor (runChannel / collBatchKernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=60000; O=gpurun_out/r02c13; rm -rf $O; mkdir -p $O/s
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 650 --timeout-method thread > $O/pytest_full.log 2>&1; rc=$?
echo "fullsize rc=$rc"; tail -8 $O/pytest_full.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { echo bench failed; exit 1; }
tail -c 400 $O/bench_n1.json; echo
CFG=scripts/cfg/n2_sweep2.json
timeout -k 10 240 python3 scripts/rank_sweep.py 1 2 $O/s $CFG > $O/s/r1.log 2>&1 &
P1=$!
timeout -k 10 240 python3 scripts/rank_sweep.py 0 2 $O/s $CFG > $O/s/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "sweep rank0=$R0 rank1=$R1"; cat $O/s/rank0.jsonl
