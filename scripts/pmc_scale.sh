#!/bin/bash
# PMC HBM passes (scripts/pmc_n2.sh) of the 256 MiB fp32 AllReduce at n = 2, 4, 8 ranks on the one GPU (rank 0
# profiled), the staged default and, at n = 2, the push gather and eager zero-copy; per-launch summary in
# gpurun_out/pmc2/summary.json (-> profiles/pmc_traffic.json: allreduce_f32_256MiB_n{2,4,8}).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for N in ${NS:-2 4 8}; do NRANKS=$N MODE=staged bash scripts/pmc_n2.sh || exit 1; done
for M in ${MODES:-push eager}; do NRANKS=2 MODE=$M bash scripts/pmc_n2.sh || exit 1; done
TAGS=""
for N in ${NS:-2 4 8}; do [ $N = 2 ] && TAGS="$TAGS staged" || TAGS="$TAGS staged_n$N"; done
python3 scripts/pmc_n2_summary.py $TAGS ${MODES:-push eager} > gpurun_out/pmc2/summary.json && cat gpurun_out/pmc2/summary.json
