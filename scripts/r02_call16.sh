#!/bin/bash
# Round 2 call 16: store-atomicity probe on one GPU (cross-XCD), window tests incl. mixed in-place ranks.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c16; rm -rf $O; mkdir -p $O
timeout -k 10 60 ./tests/native/store_atomicity_probe 0 0 20000 64 3000 > $O/probe1.json 2>&1 || { cat $O/probe1.json; exit 1; }
cat $O/probe1.json
timeout -k 10 60 ./tests/native/store_atomicity_probe 0 0 200000 8 3000 > $O/probe2.json 2>&1 || { cat $O/probe2.json; exit 1; }
cat $O/probe2.json
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_windows.py tests/test_gpu_native.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -30; tail -2 $O/pytest.log; echo "pytest rc=$rc"
