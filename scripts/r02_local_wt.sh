#!/bin/bash
# Local output stores of the staged / one-shot / symmetric kernels: global nontemporal (default build) vs
# system-scope write-through buffer stores (ablib/lwt, -DNCCL_AMD_LOCAL_WT=1), n=2 one-GPU rehearsal,
# alternating builds; then bench.py N=1 (default copy = write-through buffer stores) once.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/lwt; rm -rf $O; mkdir -p $O
i=0
for L in nccl_amd/lib/libnccl.so ablib/lwt/libnccl.so nccl_amd/lib/libnccl.so ablib/lwt/libnccl.so; do
  i=$((i+1)); D=$O/run$i; mkdir -p $D
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 1 2 $D scripts/cfg/ab_refactor.json > $D/r1.log 2>&1 &
  P1=$!
  NCCL_AMD_LIB=$PWD/$L timeout -k 10 200 python3 scripts/rank_sweep.py 0 2 $D scripts/cfg/ab_refactor.json > $D/r0.log 2>&1; R0=$?
  wait $P1; R1=$?
  echo "run $i $L rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { tail -5 $D/r0.log $D/r1.log; exit 1; }
  python3 -c "import json,sys; [print(' ', d['name'], d['ms'], d['check']) for d in map(json.loads, open('$D/rank0.jsonl'))]"
done
