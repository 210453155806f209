#!/bin/bash
# NCCL_AMD_REF_ORDER on the reference's RING/LL and RING/LL128 partitions: multi-process cases, golden fixtures,
# C4's full-size columns, then a short fuzz with the protocol buffer knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/ref_proto; rm -rf $O; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_collectives.py -k "REF_ORDER or RING" > $O/pytest_coll.log 2>&1; rc=$?
tail -n 2 $O/pytest_coll.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 $PYT tests/test_gpu_golden.py > $O/pytest_golden.log 2>&1; rc=$?
tail -n 2 $O/pytest_golden.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 $PYT tests/test_gpu_fullsize.py -k c4 > $O/pytest_c4.log 2>&1; rc=$?
tail -n 2 $O/pytest_c4.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -u scripts/fuzz.py 120 41 > $O/fuzz.log 2>&1; rc=$?
tail -n 2 $O/fuzz.log; exit $rc
