#!/bin/bash
# Round 3: the reference's ring partition (NCCL_ALGO=RING) on the GPU first, then the full check (scripts/gpu_full.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 300 $PYT tests/test_gpu_collectives.py -k "ring or RING" > gpurun_out/pytest_ring.log 2>&1 && echo RING_OK &&
timeout -k 10 300 $PYT tests/test_gpu_golden.py > gpurun_out/pytest_golden.log 2>&1 && echo GOLDEN_OK &&
bash scripts/gpu_full.sh
tail -3 gpurun_out/pytest_ring.log gpurun_out/pytest_golden.log
