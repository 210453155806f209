#!/bin/bash
# Forced ring on the LL / LL128 partitions: ring and reference-order cases, golden fixtures, short fuzz.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/ring_proto; rm -rf $O; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_collectives.py -k "REF_ORDER or RING or ring" > $O/pytest_coll.log 2>&1; rc=$?
tail -n 2 $O/pytest_coll.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 $PYT tests/test_gpu_golden.py > $O/pytest_golden.log 2>&1; rc=$?
tail -n 2 $O/pytest_golden.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -u scripts/fuzz.py 120 43 > $O/fuzz.log 2>&1; rc=$?
tail -n 2 $O/fuzz.log; exit $rc
