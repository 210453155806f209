#!/bin/bash
# Round 2 call 10: group batching (staged + widened LL) on the GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_api.py \
  > gpurun_out/r02_call10_api.log 2>&1
