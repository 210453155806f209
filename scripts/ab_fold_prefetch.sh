#!/bin/bash
# A/B: foldRange with (this build) and without (abvar/nopf, -DNCCL_AMD_FOLD_PREFETCH=0) the next batch's first
# source loaded during the last source's fold; n-process 256 MiB fp32 AllReduce on the one GPU (scripts/mp_rank.py,
# rank 0's event time per AllReduce), eager zero-copy and staged at n = 2 and 8, builds interleaved over 3 rounds.
# Build the variant first: make lib EXTRA=-DNCCL_AMD_FOLD_PREFETCH=0 BUILD=build_ab_nopf LIBDIR=abvar/nopf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
O=gpurun_out/ab_pf; rm -rf $O; mkdir -p $O
for ROUND in 1 2 3; do
  for L in abvar/nopf/libnccl.so nccl_amd/lib/libnccl.so; do
    for M in eager staged; do
      for N in 2 8; do
        U=/tmp/uid_ab_${ROUND}_${M}_$N.bin; rm -f $U
        export NRANKS=$N NCCL_AMD_LIB=$PWD/$L
        PIDS=""
        for R in $(seq 1 $((N - 1))); do
          timeout -k 5 120 python3 scripts/mp_rank.py $R $U 20 $M > $O/r${R}.log 2>&1 &
          PIDS="$PIDS $!"
        done
        timeout -k 5 120 python3 scripts/mp_rank.py 0 $U 20 $M > $O/r0.log 2>&1; R0=$?
        RP=0; for P in $PIDS; do wait $P || RP=$?; done
        [ $R0 -eq 0 ] && [ $RP -eq 0 ] || { echo "FAIL $L $M $N"; cat $O/r0.log; exit 1; }
        echo "round $ROUND $(basename $(dirname $L)) $M n=$N $(grep -o 'ok=[A-Za-z]* async=[0-9]* ms=[0-9.]*' $O/r0.log)"
      done
    done
  done
done
