#!/bin/bash
# Round 2 call 17: LL128-class (LL64) protocol parity + latency vs LL / one-shot on the one-GPU box.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c17; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_collectives.py \
  -k "ll128 or ll_and_ll128 or LL128 or ll_epoch or ll_reducescatter" tests/test_gpu_windows.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -30; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
for P in "LL" "LL128" "^LL" ; do
  for G in 0 1; do
    NCCL_PROTO=$P timeout -k 10 60 ./tests/native/nccl_perf -r 2 -b 8 -e 1048576 -f 2 -i 100 -w 10 -g $G > $O/perf_${P}_g$G.txt 2>&1 || { cat $O/perf_${P}_g$G.txt; exit 1; }
    echo "== proto $P graph $G"; grep -v "^#" $O/perf_${P}_g$G.txt | awk '{printf "%s:%s(%s) ", $1, $3, $6}'; echo
  done
done
