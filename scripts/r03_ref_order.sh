#!/bin/bash
# NCCL_AMD_REF_ORDER: parity (multi-process ring / reference-order cases, golden ring fixtures, forced ring/tree)
# then its rate against the default direct kernel and the ring (n = 2 and 4 on the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/ref_order; rm -rf $O; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_collectives.py -k "RING or REF_ORDER or ring" > $O/pytest_coll.log 2>&1; rc=$?
tail -n 2 $O/pytest_coll.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 $PYT tests/test_gpu_golden.py > $O/pytest_golden.log 2>&1; rc=$?
tail -n 2 $O/pytest_golden.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u scripts/ref_order_rate.py 256 10 > $O/rate.jsonl 2>&1; rc=$?
cat $O/rate.jsonl | grep '^{'; exit $rc
