#!/bin/bash
# Reference-order parity + rate on the one-GPU box (n = 2 rehearsal): the parity tests of the reference-partition
# paths, the rate of every mode (REPS interleaved rounds each, median / min / max; both starting orders), then a kernel trace of the default direct kernel against the
# reference-order kernel at K = 32 alone (collKernel<float,0,0> vs collKernel<float,0,5>).
# Usage: gpurun -- 'bash scripts/ref_order_ab.sh [TAG]'   (output under gpurun_out/ref_ab_TAG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/ref_ab_${1:-run}; rm -rf $O; mkdir -p $O
export NCCL_AMD_SPIN_TIMEOUT_MS=30000
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_collectives.py::test_multi_process \
  "tests/test_gpu_api.py::test_hipgraph_reference_order_allreduce" "tests/test_gpu_fullsize.py::test_c4_allreduce_fp16_sweep_every_algorithm_n8" \
  -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -cE "PASSED" $O/pytest.log; tail -2 $O/pytest.log
fi
NS=2 timeout -k 10 300 python3 -u scripts/ref_order_rate.py 256 30 > $O/fwd.jsonl 2>&1 &&
NS=2 REVERSE=1 timeout -k 10 300 python3 -u scripts/ref_order_rate.py 256 30 > $O/rev.jsonl 2>&1 &&
NS=2 MODES_SEL=direct,ref_order_k32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python3 -u scripts/ref_order_rate.py 256 20 > $O/prof.log 2>&1
rc=$?; grep -h '^{' $O/fwd.jsonl $O/rev.jsonl; find $O/prof -name "*kernel_stats.csv" | head -3; exit $rc
