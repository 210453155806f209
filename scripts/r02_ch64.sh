#!/bin/bash
# Anatomy of the 64-channel n=2 rehearsal (256 MiB fp32 AllReduce): steps per channel (slot size), slot count,
# pull variants, no-acquire; ch256 for reference (scripts/cfg/ch64_anatomy.json).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/ch64; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 scripts/rank_sweep.py 1 2 $O scripts/cfg/ch64_anatomy.json > $O/r1.log 2>&1 &
P1=$!
timeout -k 10 300 python3 scripts/rank_sweep.py 0 2 $O scripts/cfg/ch64_anatomy.json > $O/r0.log 2>&1; R0=$?
wait $P1; R1=$?
echo "rank0=$R0 rank1=$R1"; [ $R0 -eq 0 ] && [ $R1 -eq 0 ] || { tail -5 $O/r0.log $O/r1.log; exit 1; }
python3 -c "import json; [print(' ', d['name'], d['ms'], d['check']) for d in map(json.loads, open('$O/rank0.jsonl'))]"
