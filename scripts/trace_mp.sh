#!/bin/bash
# rocprofv3 kernel trace (--stats) of rank 0 of an n-process 256 MiB fp32 AllReduce on the one GPU (scripts/mp_rank.py,
# ranks 1..n-1 plain processes), for MODE (staged | eager) at each N in NS. Outputs: gpurun_out/trace_mp/<mode>_n<N>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
mkdir -p gpurun_out/trace_mp
for M in ${MODES:-eager staged}; do
  for N in ${NS:-2 8}; do
    U=/tmp/uid_trace_${M}_$N.bin; rm -f $U
    export NRANKS=$N
    PIDS=""
    for R in $(seq 1 $((N - 1))); do
      timeout -k 5 120 python3 scripts/mp_rank.py $R $U 20 $M > gpurun_out/trace_mp/rank${R}_${M}_n$N.log 2>&1 &
      PIDS="$PIDS $!"
    done
    timeout -k 10 110 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_mp/${M}_n$N -o run -- \
      python3 scripts/mp_rank.py 0 $U 20 $M > gpurun_out/trace_mp/rank0_${M}_n$N.log 2>&1
    R0=$?
    RP=0
    for P in $PIDS; do wait $P || RP=$?; done
    echo "$M n=$N rank0=$R0 peers=$RP"
    if [ $R0 -ne 0 ] || [ $RP -ne 0 ]; then exit 1; fi
  done
done
