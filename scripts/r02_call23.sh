#!/bin/bash
# Round 2 call 23: inline-asm remote stores (ablib/asm) vs compiler-visible buffer stores (default build):
# n=2 rehearsal channel sweep, then the collective parity tests on the buffer-store build.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c23; rm -rf $O; mkdir -p $O
i=0
for L in ablib/asm/libnccl.so nccl_amd/lib/libnccl.so ablib/asm/libnccl.so nccl_amd/lib/libnccl.so; do
  i=$((i+1)); D=$O/run$i; mkdir -p $D
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 1 2 $D > $D/r1.log 2>&1 &
  P1=$!
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 0 2 $D > $D/r0.log 2>&1; R0=$?
  wait $P1; R1=$?
  echo "run $i $L rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { tail -5 $D/r0.log $D/r1.log; exit 1; }
  python3 -c "import json,sys; [print(' ', d['name'], d['ms'], d['check']) for d in map(json.loads, open('$D/rank0.jsonl'))]"
done
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_collectives.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | tail -10; tail -2 $O/pytest.log; echo "pytest rc=$rc"
