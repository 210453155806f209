#!/bin/bash
# Round 2 call 15: IPC fallback / legacy cases, windows (2 GiB) and multi-process suites after the ipc.cc change.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c15; rm -rf $O; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_collectives.py tests/test_gpu_windows.py -k "multi_process or two_gib" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -30; tail -2 $O/pytest.log; echo "pytest rc=$rc"
