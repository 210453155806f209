#!/bin/bash
# Round 3: n=2 one-GPU AllReduce rate per element type / operator (scripts/dtype_rate.py, 256 MiB per rank),
# staged and registered, for this build and the 1-byte-fold variant in ablib/v1 (A, B, A, B), then the roctx
# marker trace (scripts/r03_roctx.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
D=gpurun_out/r03dtype
mkdir -p $D
i=0
for L in nccl_amd/lib/libnccl.so ablib/v1/libnccl.so nccl_amd/lib/libnccl.so ablib/v1/libnccl.so; do
  i=$((i+1))
  for M in staged reg; do
    NCCL_AMD_LIB=$PWD/$L MODE=$M timeout -k 10 300 python3 scripts/dtype_rate.py 256 20 > $D/run${i}_$M.jsonl 2> $D/run${i}_$M.err \
      || { echo "run $i $L $M failed"; tail -3 $D/run${i}_$M.err; exit 1; }
    echo "run $i $L $M ok"
  done
done
bash scripts/r03_roctx.sh
