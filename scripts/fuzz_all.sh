#!/bin/bash
# Randomized parity fuzz (scripts/fuzz.py: knob mix incl. LL128, windows, registered buffers, fence, CU budget):
# single process for FUZZ_SECS (default 240), then 2-4 processes (scripts/fuzz_mp.py). SEED picks the sequence.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/fuzz; rm -rf $O; mkdir -p $O
S=${SEED:-22}
timeout -k 10 $(( ${FUZZ_SECS:-240} + 60 )) python3 -u scripts/fuzz.py ${FUZZ_SECS:-240} $S > $O/fuzz.log 2>&1; rc=$?
tail -3 $O/fuzz.log; echo "fuzz rc=$rc"; [ $rc -eq 0 ] || exit 1
for N in 2 3 4; do
  timeout -k 10 300 python3 -u scripts/fuzz_mp.py $N 12 $((S * 10 + N)) > $O/fuzz_mp$N.log 2>&1; rc=$?
  tail -2 $O/fuzz_mp$N.log; echo "fuzz_mp $N rc=$rc"; [ $rc -eq 0 ] || exit 1
done
