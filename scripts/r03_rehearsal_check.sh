#!/bin/bash
# After the caller-thread release fix: the driver's multi-GPU bench command at N=4 (the failing case: a
# deregistration, then new communicators) and N=2 on the one GPU, with suite tracing; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/rehearsal_check; rm -rf $O; mkdir -p $O
for N in 4 2; do
  BENCH_TRACE=1 NCCL_DEBUG=WARN timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29760 + N)) bench.py --gpus $N --steps 20 --warmup 5 > $O/bench_n$N.log 2>&1
  rc=$?; echo "N=$N rc=$rc"
  grep -E "WARN|rror" $O/bench_n$N.log | grep -v amdgpu.ids | head -20
  grep '^{"metric"' $O/bench_n$N.log > $O/bench_n$N.json
  python3 - $O/bench_n$N.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
s = d.get("suite", {})
print("value", d["value"], "check", d["check"], "suite s", s.get("seconds"), "err", s.get("error"))
for k, v in s.items():
    if isinstance(v, dict) and "check" in v:
        print(" ", k, v["check"])
st = s.get("staged_tuning", {}).get("runs", [])
print("  staged_tuning", sum(r["check"].startswith("pass") for r in st), "of", len(st), "pass")
PY
  [ $rc -eq 0 ] || exit 1
done
