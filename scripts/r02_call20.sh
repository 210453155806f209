#!/bin/bash
# Round 2 call 20: packs in flight per thread vs channel count (n=2 rehearsal, 256 MiB fp32): default build
# (copy 8 / fold 4), copy 16 / fold 4, copy 16 / fold 6; channels 256/128/64/32, alternating builds.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c20; rm -rf $O; mkdir -p $O
i=0
for L in nccl_amd/lib/libnccl.so ablib/c16/libnccl.so ablib/c16f6/libnccl.so nccl_amd/lib/libnccl.so ablib/c16/libnccl.so ablib/c16f6/libnccl.so; do
  i=$((i+1)); D=$O/run$i; mkdir -p $D
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 1 2 $D > $D/r1.log 2>&1 &
  P1=$!
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 0 2 $D > $D/r0.log 2>&1; R0=$?
  wait $P1; R1=$?
  echo "run $i $L rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { tail -5 $D/r0.log $D/r1.log; exit 1; }
  python3 -c "import json,sys; [print(' ', d['name'], d['ms'], d['check']) for d in map(json.loads, open('$D/rank0.jsonl'))]"
done
