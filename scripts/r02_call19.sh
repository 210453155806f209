#!/bin/bash
# Round 2 call 19: window tests (mixed in-place AllGather), LL128 multi-process size table, and the
# direct path's channel granularity at mid sizes (n=2, n=4 on one GPU).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/r02c19; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_windows.py \
  "tests/test_gpu_collectives.py::test_multi_process[n4-LL128=1]" tests/test_gpu_native.py::test_store_atomicity_probe_one_gpu > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -30; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
run() { timeout -k 10 90 ./tests/native/nccl_perf -r $1 -b 262144 -e 67108864 -f 4 -i 30 -w 5 -g 1 > $O/p.txt 2>&1 || { cat $O/p.txt; exit 1; }
        echo "$2 r=$1: $(grep -v '^#' $O/p.txt | awk '{printf "%s:%s(%s) ", $1, $3, $6}')"; }
for R in 2 4; do
  for MB in 65536 32768 16384 8192; do NCCL_ALGO=DIRECT NCCL_PROTO=Simple NCCL_AMD_MIN_CHANNEL_BYTES=$MB run $R "direct mcb=$MB"; done
  for MB in 16384 4096; do NCCL_ALGO=ONESHOT NCCL_PROTO=Simple NCCL_AMD_ONESHOT_CHANNEL_BYTES=$MB run $R "oneshot ocb=$MB"; done
done
