#!/bin/bash
# Round 3: FETCH_SIZE / WRITE_SIZE of the n=2 AllReduce kernels, 256 MiB fp32 per rank, one process per rank
# on the one GPU (rank 0 under rocprofv3 --pmc, rank 1 plain: a profiled process serialises its own kernels, so
# both ranks in one profiled process would deadlock) — registered (ncclCommRegister) and symmetric-window modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for M in reg sym; do MODE=$M bash scripts/pmc_n2.sh || exit 1; done
