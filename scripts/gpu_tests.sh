#!/bin/bash
# GPU-box run of the parity suite (one pytest process; time-limited; per-test timeout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 1000 python -m pytest tests -m gpu -v -s --timeout 240 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
grep -E "PASSED|FAILED|mismatch|Timeout" gpurun_out/pytest_gpu.log | cut -c1-400 | head -40
