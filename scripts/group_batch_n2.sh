#!/bin/bash
# group batching across processes + aggregated vs unaggregated group timing (n=2, one GPU).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c11; rm -rf $O; mkdir -p $O/g
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_api.py -k "batches or aggregates" > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
CFG=scripts/cfg/group_batch.json
timeout -k 10 240 python3 scripts/rank_sweep.py 1 2 $O/g $CFG > $O/g/r1.log 2>&1 &
P1=$!
timeout -k 10 240 python3 scripts/rank_sweep.py 0 2 $O/g $CFG > $O/g/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "sweep rank0=$R0 rank1=$R1"; cat $O/g/rank0.jsonl
