#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 900 python -m pytest tests/test_gpu_collectives.py -v -s -k multi_process > gpurun_out/pytest_mp.log 2>&1 && echo PYTEST_OK
