#!/bin/bash
# Store cache policy of the nRanks==1 copy: the probe (scripts/copy_policy_probe.hip), then bench.py N=1 with
# each library variant (NCCL_AMD_COPY_VARIANT: 0 global nt store, 4 buffer sc0|sc1, 5 sc1, 6 sc1|nt, 7 nt),
# alternating so box drift shows. Each step time-limited; stop at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/store_policy; rm -rf $O; mkdir -p $O
timeout -k 10 120 ./scripts/copy_policy_probe > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
for v in 0 4 5 6 7 0 4 5; do
  NCCL_AMD_COPY_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra > $O/bench_v$v.log 2>&1 || { tail -5 $O/bench_v$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_v$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['check'])"
done
