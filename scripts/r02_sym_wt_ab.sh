#!/bin/bash
# Symmetric-window AllReduce (n=2, both ranks in one process on the one GPU, 256 MiB fp32 per rank):
# publish with the default nontemporal stores + L2 write-back release (NCCL_AMD_SYM_WT=0) vs system-scope
# write-through stores + store drain only (NCCL_AMD_SYM_WT=1), alternating, three runs each; then the
# symmetric-window parity tests under NCCL_AMD_SYM_WT=1. Every step time-limited; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/symwt; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for W in 0 1; do
    NCCL_AMD_SYM_WT=$W MODE=sym STEPS=50 timeout -k 10 120 python3 scripts/multirank_one_gpu.py > $O/sym_wt${W}_$i.log 2>&1 \
      || { echo "sym wt=$W run $i failed"; tail -5 $O/sym_wt${W}_$i.log; exit 1; }
    echo "wt=$W run $i $(tail -1 $O/sym_wt${W}_$i.log)"
  done
done
NCCL_AMD_SYM_WT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_windows.py -x -q --timeout 240 --timeout-method thread \
  > $O/windows_wt1.log 2>&1 || { tail -20 $O/windows_wt1.log; exit 1; }
tail -1 $O/windows_wt1.log
echo SYMWT_OK
