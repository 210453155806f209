#!/bin/bash
# Round 6 PMC passes (scripts/pmc_n2.sh) of the 256 MiB fp32 AllReduce on the one GPU, rank 0 profiled: the staged
# kernel at n = 2, 4, 8 (the per-channel peer order must leave its bytes unchanged) and eager zero-copy (the
# multi-process default since round 6) at n = 2, 4, 8. Summary: gpurun_out/pmc2/summary_r06.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for N in 2 4 8; do NRANKS=$N MODE=staged bash scripts/pmc_n2.sh || exit 1; done
for N in 2 4 8; do NRANKS=$N MODE=eager bash scripts/pmc_n2.sh || exit 1; done
python3 scripts/pmc_n2_summary.py staged staged_n4 staged_n8 eager eager_n4 eager_n8 > gpurun_out/pmc2/summary_r06.json \
  && cat gpurun_out/pmc2/summary_r06.json
