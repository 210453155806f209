#!/bin/bash
# PMC HBM counters of the n-rank staged AllReduce kernel (256 MiB per rank; NRANKS, default 2): rank 0 under
# rocprofv3, ranks 1..n-1 plain processes (separate passes for FETCH_SIZE and WRITE_SIZE). Outputs go to
# gpurun_out/pmc2/<mode>[_n<N>]_<counter>/ (scripts/pmc_n2_summary.py reads them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
mkdir -p gpurun_out/pmc2
M=${MODE:-staged}
N=${NRANKS:-2}
export NRANKS=$N
TAG=$M; [ "$N" != 2 ] && TAG=${M}_n$N
for C in FETCH_SIZE WRITE_SIZE; do
  U=/tmp/uid_$C.bin; rm -f $U
  PIDS=""
  for R in $(seq 1 $((N - 1))); do
    timeout -k 5 120 python3 scripts/mp_rank.py $R $U 5 $M > gpurun_out/pmc2/rank${R}_${TAG}_$C.log 2>&1 &
    PIDS="$PIDS $!"
  done
  timeout -s KILL 110 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc2/${TAG}_$C -o run -- python3 scripts/mp_rank.py 0 $U 5 $M \
    > gpurun_out/pmc2/rank0_${TAG}_$C.log 2>&1
  R0=$?
  RP=0
  for P in $PIDS; do wait $P || RP=$?; done
  echo "$C n=$N rank0=$R0 peers=$RP"
  if [ $R0 -ne 0 ] || [ $RP -ne 0 ]; then exit 1; fi
done
