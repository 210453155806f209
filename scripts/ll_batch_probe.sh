# LL group-batch probe: device time of G small AllReduces in one group (tests/native/nccl_perf -G), two ranks
# on one GPU, and the group / LL GPU tests. usage: bash scripts/ll_batch_probe.sh [sweep|test]
set -e
mkdir -p gpurun_out
export NCCL_MULTI_RANK_GPU_ENABLE=1 NCCL_AMD_FORK_JOIN=0
if [ "${1:-sweep}" = sweep ]; then
  for G in 1 8 16 32; do
    echo "G=$G"; timeout -k 10 60 tests/native/nccl_perf -d 1 -r 2 -b 4096 -e 4096 -t half -i 200 -w 20 -G $G -H 1
  done > gpurun_out/llg_sweep.txt 2>&1
  timeout -k 10 60 tests/native/nccl_perf -d 1 -r 2 -b 131072 -e 131072 -t half -i 200 -w 20 -H 1 >> gpurun_out/llg_sweep.txt 2>&1
fi
unset NCCL_AMD_FORK_JOIN
NCCL_DEBUG=TRACE timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_api.py -k "group_defers or mixed_coll" > gpurun_out/llg_trace.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_api.py \
  tests/test_gpu_collectives.py -k "group or aggregat or batch or ll or fuzz" > gpurun_out/llg_pytest.txt 2>&1
