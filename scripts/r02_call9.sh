#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r02c9; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_collectives.py tests/test_gpu_windows.py -k "ring_and_tree or RING or TREE or single_process or windows" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -25; echo "pytest rc=$rc"
