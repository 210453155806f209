#!/bin/bash
# which bench.py part order makes the N = 2 rehearsal's small collectives slow (27.6 us instead
# of 4.2), and why. Each run: torchrun N=2 on the one GPU, quick suite, host-staged part first (BENCH_HOST_STAGED=
# first), only the parts named; prints the fp16 sweep's 8 B .. 2 KiB LL / default columns. Then a traced run.
# Usage: gpurun -- 'bash scripts/order_probe.sh [TAG]'   (output under gpurun_out/order_TAG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/order_${1:-run}; rm -rf $O; mkdir -p $O
export NCCL_AMD_SPIN_TIMEOUT_MS=20000 BENCH_SWEEP_COLS=ll,default
run() {  # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 --steps 3 --warmup 1 --quick-suite --no-cpu-baseline \
    > $O/$name.log 2>&1 || { echo "$name FAILED"; tail -5 $O/$name.log; return 1; }
  python3 - "$name" "$O/$name.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
rows = d.get("suite", {}).get("ar_fp16_sweep", [])
print(sys.argv[1], [(r["bytes"], r.get("ll_us"), r.get("default_us")) for r in rows[:5]])
PY
}
run base BENCH_SUITE_PARTS=ar_fp16_sweep &&
run first_sweep BENCH_HOST_STAGED=first BENCH_SUITE_PARTS=ar_fp16_sweep &&
run first_rsag_sweep BENCH_HOST_STAGED=first BENCH_SUITE_PARTS=rs_ag_bf16,ar_fp16_sweep &&
run first_nopipe_rsag_sweep BENCH_HOST_STAGED=first BENCH_HOST_STAGED_PIPE=0 BENCH_SUITE_PARTS=rs_ag_bf16,ar_fp16_sweep &&
run rsag_sweep BENCH_SUITE_PARTS=rs_ag_bf16,ar_fp16_sweep
