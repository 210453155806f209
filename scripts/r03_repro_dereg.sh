#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dereg; export TMPDIR=/tmp
for M in bench nodereg barrier; do
  timeout -k 10 200 python3 -u scripts/repro_dereg.py 4 $M > gpurun_out/dereg/$M.log 2>&1; rc=$?
  tail -n 1 gpurun_out/dereg/$M.log; echo "$M rc=$rc"; [ $rc -eq 0 ] || exit 1
done
