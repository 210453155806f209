#!/bin/bash
# Smoke + the symmetric-window and API GPU tests on the final build (every step time-limited, stop at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/win; export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/win/smoke.log 2>&1 || { tail gpurun_out/win/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 600 python -u -m pytest tests/test_gpu_windows.py tests/test_gpu_native.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/win/pytest.log 2>&1 || { grep -E "FAILED|ERROR" gpurun_out/win/pytest.log | tail; tail -3 gpurun_out/win/pytest.log; exit 1; }
tail -1 gpurun_out/win/pytest.log
echo WIN_OK  # then a fuzz run with window cases
timeout -k 10 240 python3 -u scripts/fuzz.py 150 47 > gpurun_out/win/fuzz.log 2>&1 || { tail -5 gpurun_out/win/fuzz.log; exit 1; }
grep -c "window\|SYM_WT" gpurun_out/win/fuzz.log || true
tail -2 gpurun_out/win/fuzz.log
echo WINFUZZ_OK
