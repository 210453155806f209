#!/bin/bash
# Round 2 call 12: smoke + the whole GPU suite except the full-size configs (those run in call 13).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r02c12; rm -rf $O; mkdir -p $O
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  --ignore=tests/test_gpu_fullsize.py > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -3 $O/pytest_gpu.log; exit $rc
