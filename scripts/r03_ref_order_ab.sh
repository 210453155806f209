#!/bin/bash
# A/B of the direct kernel vs the reference-order kernel at n = 2 (one GPU), both mode orders, then a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/ref_ab; rm -rf $O; mkdir -p $O
NS=2 timeout -k 10 200 python3 -u scripts/ref_order_rate.py 256 50 > $O/fwd.jsonl 2>&1 &&
NS=2 REVERSE=1 timeout -k 10 200 python3 -u scripts/ref_order_rate.py 256 50 > $O/rev.jsonl 2>&1 &&
NS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u scripts/ref_order_rate.py 256 20 > $O/prof.log 2>&1
rc=$?; grep -h '^{' $O/fwd.jsonl $O/rev.jsonl; exit $rc
