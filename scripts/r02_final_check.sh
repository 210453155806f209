#!/bin/bash
# End-of-session check of the final build: smoke, the full GPU suite, a 2-minute single-process fuzz and
# 2- and 4-process fuzz runs. Every step bounded; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/final; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK || { tail $O/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u scripts/fuzz.py 120 31 > $O/fuzz.log 2>&1 || { tail -5 $O/fuzz.log; exit 1; }
tail -2 $O/fuzz.log
for N in 2 4; do
  timeout -k 10 200 python3 -u scripts/fuzz_mp.py $N 8 $((310 + N)) > $O/fuzz_mp$N.log 2>&1 || { tail -5 $O/fuzz_mp$N.log; exit 1; }
  tail -1 $O/fuzz_mp$N.log
done
echo FINAL_OK
