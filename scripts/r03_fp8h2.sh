#!/bin/bash
# Round 3: the packed-half fp8 fold. Probe, 1-byte parity (every code pair, every operator, LL and staged; fp8
# special values), then the n=2 rate A/B against the f32-path build in abvar/h0 (A, B, A, B), fp8 / u8 / f32 rows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp NCCL_AMD_SPIN_TIMEOUT_MS=20000
D=gpurun_out/r03fp8h2; mkdir -p $D
timeout -k 5 60 tests/native/fp8_f16_probe > $D/probe.json 2>&1 && cat $D/probe.json &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_numerics.py \
  > $D/pytest_numerics.log 2>&1 && echo NUMERICS_OK &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_collectives.py \
  -k "special or single_process or one_byte" > $D/pytest_coll.log 2>&1 && echo COLL_OK || { tail -5 $D/*.log; exit 1; }
i=0
for L in nccl_amd/lib/libnccl.so abvar/h0/libnccl.so nccl_amd/lib/libnccl.so abvar/h0/libnccl.so; do
  i=$((i+1))
  for M in staged reg; do
    NCCL_AMD_LIB=$PWD/$L MODE=$M timeout -k 10 300 python3 scripts/dtype_rate.py 256 20 > $D/run${i}_$M.jsonl 2> $D/run${i}_$M.err \
      || { echo "run $i $L $M failed"; tail -3 $D/run${i}_$M.err; exit 1; }
    echo "run $i $L $M ok"
  done
done
