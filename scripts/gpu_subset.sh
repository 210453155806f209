#!/bin/bash
# GPU-box run of a pytest selection (args: pytest node ids / -k expressions), time-limited, log under gpurun_out/.
# Usage: gpurun -- 'bash scripts/gpu_subset.sh NAME tests/test_x.py ...'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
name=$1; shift
export NCCL_AMD_SPIN_TIMEOUT_MS=${NCCL_AMD_SPIN_TIMEOUT_MS:-20000}
timeout -k 10 ${SUBSET_TIMEOUT:-900} python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/$name.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/$name.log | tail -40
tail -3 gpurun_out/$name.log
exit $rc
