#!/bin/bash
# A/B of nRanks==1 copy variants through bench.py at N=1, alternating on one box: value, launch average, warm and
# cold (rotated buffers) fraction per run. Each entry of VARIANTS is V or V:S (NCCL_AMD_COPY_VARIANT=V,
# NCCL_AMD_COPY_XCD_SHIFT=S). VARIANTS="10 0" REPS=3 by default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
  for vs in ${VARIANTS:-10 0}; do
    v=${vs%%:*}; sh=12; [[ $vs == *:* ]] && sh=${vs##*:}
    NCCL_AMD_COPY_VARIANT=$v NCCL_AMD_COPY_XCD_SHIFT=$sh timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      > gpurun_out/copy_ab_${v}_${sh}_${rep}.log 2>&1 || { echo "variant $vs rep $rep FAILED"; exit 1; }
    python3 - "$vs" gpurun_out/copy_ab_${v}_${sh}_${rep}.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
r = d["roofline"]
print(f"variant {sys.argv[1]:>5} value {d['value']:8.1f} launch_ms {r.get('launch_avg_ms')} frac {r['frac']:.4f} "
      f"frac_cold {r.get('frac_cold')} check {d['check'] if isinstance(d['check'], str) else d['check'].get('pass', d['check'])}")
PY
  done
done
