#!/bin/bash
# The round-5 co-residency setting (64 channels per rank at 8 ranks on the one GPU, NCCL_AMD_SHARED_GPU_CHANNELS=64)
# under the n = 8 tuning part, RUNS times, each rank logging WARNs: does the round-5 stall come back?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cap64
export NCCL_AMD_SPIN_TIMEOUT_MS=20000 BENCH_TRACE=1 BENCH_SUITE_PARTS=staged_tuning BENCH_NO_LINEUP=1 \
  NCCL_AMD_SHARED_GPU_CHANNELS=${CH:-64}
for RUN in $(seq 1 ${RUNS:-3}); do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29770 + RUN)) bench.py --gpus 8 --steps 10 --warmup 3 --no-cpu-baseline --no-extra \
    > gpurun_out/cap64/run$RUN.log 2>&1 || { echo "run $RUN rc=$?"; exit 1; }
  python3 - gpurun_out/cap64/run$RUN.log <<'PY'
import json, sys
t = open(sys.argv[1]).read(); i = t.find('{"metric"'); d = json.loads(t[i:].splitlines()[0])
runs = d["suite"]["staged_tuning"]["runs"]
bad = [r for r in runs if not r["check"].startswith("pass")]
print(f"run ok: check {d['check']}, {len(runs)} columns, {len(bad)} failed: {[(r['env'], r['check'][:60]) for r in bad]}; "
      f"default {runs[0]['ms']} ms; timeouts in log: {t.count('timeout')}")
PY
done
