#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r02c7; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_windows.py tests/test_gpu_collectives.py -k "multi_process or two_gib or misalign" > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python3 scripts/ipc_hang_diag.py $O/diag 4 524288 > $O/diag.log 2>&1; echo "diag rc=$?"; tail -2 $O/diag.log
grep -h "ipc:" $O/diag/trace.*.log | head -6
