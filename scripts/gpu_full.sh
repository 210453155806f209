#!/bin/bash
# GPU-box run: smoke, full parity suite, N=1 bench (each step time-limited; stop at the first failure)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench1.log 2>&1 && echo BENCH_OK
tail -3 gpurun_out/pytest_gpu.log; tail -c 3000 gpurun_out/bench1.log
