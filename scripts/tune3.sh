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
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29999 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 2 > gpurun_out/bench_n2_suite.log 2>&1; echo "suite rc=$?"
