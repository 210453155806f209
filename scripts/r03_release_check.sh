#!/bin/bash
# The caller-thread release of peers' deregistered-buffer mappings: the registration tests (incl. the new
# deregistration -> new communicator case) and the multi-process fuzz (registered buffers in the knob mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/release_check; rm -rf $O; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_register.py \
  > $O/pytest_register.log 2>&1; rc=$?; tail -n 3 $O/pytest_register.log; [ $rc -eq 0 ] || exit 1
for N in 2 3 4; do
  timeout -k 10 300 python3 -u scripts/fuzz_mp.py $N 12 $((500 + N)) > $O/fuzz_mp$N.log 2>&1; rc=$?
  tail -n 1 $O/fuzz_mp$N.log; [ $rc -eq 0 ] || exit 1
done
