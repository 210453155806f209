#!/bin/bash
# PMC HBM counters of the n=2 staged AllReduce kernel (256 MiB per rank): rank 0 under rocprofv3, rank 1 a
# plain process (separate passes for FETCH_SIZE and WRITE_SIZE). TCC counters are device-wide, so a pass
# sees both ranks' traffic while rank 0's kernel runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
mkdir -p gpurun_out/pmc2
M=${MODE:-staged}
for C in FETCH_SIZE WRITE_SIZE; do
  U=/tmp/uid_$C.bin; rm -f $U
  timeout -k 5 100 python3 scripts/mp_rank.py 1 $U 5 $M > gpurun_out/pmc2/rank1_${M}_$C.log 2>&1 &
  P1=$!
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc2/${M}_$C -o run -- python3 scripts/mp_rank.py 0 $U 5 $M \
    > gpurun_out/pmc2/rank0_${M}_$C.log 2>&1
  R0=$?
  wait $P1; R1=$?
  echo "$C rank0=$R0 rank1=$R1"
  if [ $R0 -ne 0 ] || [ $R1 -ne 0 ]; then exit 1; fi
done
