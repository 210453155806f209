#!/bin/bash
# rocprofv3 kernel traces (+ PMC FETCH/WRITE for the staged kernel) of the n=2 AllReduce kernels with both
# ranks in one process on the box's one GPU (scripts/multirank_one_gpu.py; no child processes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
for M in direct sym ll; do
  MODE=$M timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/$M -o run -- \
    python3 scripts/multirank_one_gpu.py > gpurun_out/prof2/$M.log 2>&1 || { echo "trace $M failed"; exit 1; }
  echo "trace $M ok"
done
MODE=direct timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof2/fetch -o run -- \
  python3 scripts/multirank_one_gpu.py > gpurun_out/prof2/fetch.log 2>&1 && echo FETCH_OK &&
MODE=direct timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof2/write -o run -- \
  python3 scripts/multirank_one_gpu.py > gpurun_out/prof2/write.log 2>&1 && echo WRITE_OK
