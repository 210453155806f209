#!/bin/bash
# The nRanks==1 copy with 2 packs per thread (8 KiB tiles) + write-through stores as the default: one-rank
# parity tests, bench.py N=1 A/B against the 4-pack write-through (variant 4) and the round-1/2 nontemporal
# kernel (variant 9), then the N=1 bench line and rocprofv3 kernel trace + FETCH/WRITE passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000; O=gpurun_out/u2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_collectives.py -k "one_rank" tests/test_gpu_golden.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 4 9 0 4 9; do
  NCCL_AMD_COPY_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_v$v.log 2>&1 || { tail -5 $O/bench_v$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_v$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], 'rotated4', d.get('n1_256MiB_rotated4_hbm_GBps'), '64MiB', d.get('n1_64MiB_hbm_GBps'), d['check'])"
done
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo bench failed; tail $O/bench_n1.err; exit 1; }
tail -c 1200 $O/bench_n1.json; echo
B="python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1_trace -o run -- $B > $O/n1_trace.log 2>&1 || { echo n1 trace failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/n1_fetch -o run -- $B > $O/n1_fetch.log 2>&1 || { echo n1 fetch failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/n1_write -o run -- $B > $O/n1_write.log 2>&1 || { echo n1 write failed; exit 1; }
echo N1_PROFILES_OK
