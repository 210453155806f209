#!/bin/bash
# Round 3: the packed fp8 fold and 2-pack 1-byte folds — exhaustive 1-byte pairs, special values, 1-byte full
# channel plans, single-process multirank cases, then the per-dtype rates (staged, registered).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03fp8
export NCCL_AMD_SPIN_TIMEOUT_MS=20000
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_numerics.py \
  tests/test_gpu_collectives.py -k "numerics or every_pair or probe or special_float or one_byte or single_process_multirank or one_rank_all" \
  > gpurun_out/r03fp8/pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03fp8/pytest.log | head; tail -3 gpurun_out/r03fp8/pytest.log; exit 1; }
tail -1 gpurun_out/r03fp8/pytest.log
for M in staged reg; do
  MODE=$M timeout -k 10 300 python3 scripts/dtype_rate.py 256 20 > gpurun_out/r03fp8/$M.jsonl 2> gpurun_out/r03fp8/$M.err || exit 1
done
cat gpurun_out/r03fp8/*.jsonl | cut -c1-160
