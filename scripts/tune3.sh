#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
source scripts/tune_lib.sh
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 700 python -m pytest tests -m gpu -x -v -s > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK || exit 1; fi
run default
run nofence NCCL_AMD_P2P_FENCE=0
NP=4 run np4
NP=8 run np8
STEPS=200 SIZE=1 run small1m
STEPS=200 SIZE=1 run small1m_1shot NCCL_ALGO=ONESHOT
