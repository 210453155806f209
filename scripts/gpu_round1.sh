#!/bin/bash
# GPU-box run: smoke, bench, parity tests (each step time-limited; stop at the first failure)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK &&
timeout -k 10 900 python -m pytest tests/test_gpu_collectives.py -x -q -k "one_rank or single_process" > gpurun_out/pytest1.log 2>&1 && echo PYTEST_OK
