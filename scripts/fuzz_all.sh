#!/bin/bash
# randomized parity fuzz with the LL128 class in the knob mix: single process (4 minutes),
# then 2-4 processes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r02c22; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u scripts/fuzz.py 240 22 > $O/fuzz.log 2>&1; rc=$?
tail -3 $O/fuzz.log; echo "fuzz rc=$rc"; [ $rc -eq 0 ] || exit 1
for N in 2 3 4; do
  timeout -k 10 300 python3 -u scripts/fuzz_mp.py $N 12 $((220 + N)) > $O/fuzz_mp$N.log 2>&1; rc=$?
  tail -2 $O/fuzz_mp$N.log; echo "fuzz_mp $N rc=$rc"; [ $rc -eq 0 ] || exit 1
done
