#!/bin/bash
# PMC HBM passes (scripts/pmc_n2.sh) for the n=2 ReduceScatter, AllGather, ring and reference-order AllReduce
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for M in rs ag ring reforder; do MODE=$M bash scripts/pmc_n2.sh || exit 1; done
