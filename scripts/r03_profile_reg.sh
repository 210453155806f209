#!/bin/bash
# Round 3: n=2 one-GPU rehearsal of the registered zero-copy AllReduce against the symmetric-window and staged
# kernels (256 MiB fp32 per rank, both ranks in one process): rocprofv3 kernel traces of each, then the
# FETCH_SIZE / WRITE_SIZE passes of the registered kernel (HBM bytes per launch, MI355X_MICROARCH.md recipe).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/r03reg
mkdir -p $D
for M in direct sym reg; do
  MODE=$M timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$M -o run -- \
    python3 scripts/multirank_one_gpu.py > $D/$M.log 2>&1 || { echo "trace $M failed"; tail -5 $D/$M.log; exit 1; }
  echo "trace $M ok: $(tail -1 $D/$M.log)"
done
for C in FETCH_SIZE WRITE_SIZE; do
  MODE=reg timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D/pmc_$C -o run -- \
    python3 scripts/multirank_one_gpu.py > $D/pmc_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
  echo "pmc $C ok"
done
