#!/bin/bash
# Re-run one multi-process fuzz sequence with NCCL_DEBUG=TRACE per process (diagnosing a spin timeout).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/fmp; rm -rf $O; mkdir -p $O
NCCL_DEBUG=TRACE NCCL_DEBUG_FILE=$PWD/$O/trace.%p.log timeout -k 10 300 python3 -u scripts/fuzz_mp.py ${N:-4} 12 ${SEED:-314} > $O/out.log 2>&1
echo "rc=$?"; tail -2 $O/out.log | cut -c1-1500
