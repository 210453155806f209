#!/bin/bash
# Round 3: randomized parity fuzz (ring partition in the knob mix) then one N=1 bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FUZZ_SECS=${FUZZ_SECS:-150} SEED=${SEED:-32} bash scripts/fuzz_all.sh || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_fb.log 2>&1; rc=$?; tail -c 2500 gpurun_out/bench_fb.log; exit $rc
