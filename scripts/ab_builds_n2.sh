#!/bin/bash
# A/B of the previous build (ablib/libnccl_prev.so) and this one, n=2 sweeps alternating.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c14; rm -rf $O; mkdir -p $O
CFG=scripts/cfg/ab_refactor.json
i=0
for L in ablib/libnccl_prev.so nccl_amd/lib/libnccl.so ablib/libnccl_prev.so nccl_amd/lib/libnccl.so; do
  i=$((i+1)); D=$O/run$i; mkdir -p $D
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 1 2 $D $CFG > $D/r1.log 2>&1 &
  P1=$!
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 0 2 $D $CFG > $D/r0.log 2>&1; R0=$?
  wait $P1; R1=$?
  echo "run $i $L rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || exit 1
  python3 -c "import json,sys; [print(' ', d['name'], d['ms'], d['check']) for d in map(json.loads, open('$D/rank0.jsonl'))]"
done
