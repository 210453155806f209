#!/bin/bash
# Round 3 full check: fp8 conversion probe, smoke, full GPU suite, N=1 bench (each step time-limited).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 5 60 tests/native/fp8_cvt_probe > gpurun_out/fp8_cvt_probe.json 2>&1; echo "fp8 probe rc=$?: $(cat gpurun_out/fp8_cvt_probe.json)"
bash scripts/gpu_full.sh
