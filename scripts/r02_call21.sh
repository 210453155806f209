#!/bin/bash
# Round 2 call 21: LL64 with its own payloads preloaded before the wait: parity + latency vs LL.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c21; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_collectives.py \
  -k "ll128 or ll_and_ll128 or LL128" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -30; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
run() { timeout -k 10 60 ./tests/native/nccl_perf -r $1 -b 8 -e 1048576 -f 4 -i 100 -w 10 -g 1 > $O/p.txt 2>&1 || { cat $O/p.txt; exit 1; }
        echo "$2 r=$1: $(grep -v '^#' $O/p.txt | awk '{printf "%s:%s(%s) ", $1, $3, $6}')"; }
for R in 2 4; do for k in 1 2; do NCCL_PROTO=LL run $R "LL   "; NCCL_PROTO=LL128 run $R "LL128"; done; done
