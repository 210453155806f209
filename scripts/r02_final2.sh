#!/bin/bash
# Final check of the round-2 build with the write-through symmetric publish: smoke, full GPU suite, N=1 bench,
# then the n=2 rocprofv3 traces (staged, symmetric, LL) + FETCH/WRITE of the staged kernel (scripts/profile_n2.sh).
# Every GPU step time-limited; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | tail; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench1.log 2>&1 || { tail -5 gpurun_out/bench1.log; exit 1; }
echo BENCH_OK
bash scripts/profile_n2.sh && echo FINAL2_OK
