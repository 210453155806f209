#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c8; rm -rf $O; mkdir -p $O/plain
CFG=scripts/cfg/n2_sweep2.json
timeout -k 10 240 python3 scripts/rank_sweep.py 1 2 $O/plain $CFG > $O/plain/r1.log 2>&1 &
P1=$!
timeout -k 10 240 python3 scripts/rank_sweep.py 0 2 $O/plain $CFG > $O/plain/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "sweep rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || exit 1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_collectives.py -k "misalign or single_process" > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -5 $O/pytest.log
timeout -k 10 150 python3 scripts/ipc_hang_diag.py $O/diag 4 524288 > $O/diag.log 2>&1; echo "diag rc=$?"; tail -1 $O/diag.log
grep -h "ipc:" $O/diag/trace.*.log | head -4
