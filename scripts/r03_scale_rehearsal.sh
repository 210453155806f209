#!/bin/bash
# Round 3: the driver's multi-GPU bench command, rehearsed on the one-GPU box with the FULL suite (not --quick-suite):
# N=2 and N=4 ranks share cuda:0. Checks that every suite part finishes inside the watchdog and reports
# "pass", and records how long the suite takes. Every step time-limited; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/scale_rehearsal_r03; rm -rf $O; mkdir -p $O
for N in 2 4; do
  t0=$(date +%s)
  timeout -k 10 420 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29710 + N)) bench.py --gpus $N --steps 20 --warmup 5 > $O/bench_n$N.log 2>&1 \
    || { echo "N=$N failed rc=$?"; tail -20 $O/bench_n$N.log; exit 1; }
  echo "N=$N wall $(( $(date +%s) - t0 )) s"
  grep '^{"metric"' $O/bench_n$N.log > $O/bench_n$N.json
  python3 - $O/bench_n$N.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
s = d.get("suite", {})
print("value", d["value"], "ms", d["ms_per_step"], "check", d["check"], "suite s", s.get("seconds"), "err", s.get("error"))
for k, v in s.items():
    if isinstance(v, dict) and "check" in v:
        print(" ", k, v["check"])
EOF
done
echo REHEARSAL_OK
