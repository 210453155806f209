#!/bin/bash
# Diagnose the N=4 rehearsal stall: the driver's multi-GPU command at N=4 on the one GPU with per-part suite
# tracing, a 15 s spin timeout and NCCL_DEBUG=WARN (which rank reports what).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/rehearsal_n4_diag; rm -rf $O; mkdir -p $O
BENCH_TRACE=1 NCCL_AMD_SPIN_TIMEOUT_MS=15000 NCCL_DEBUG=WARN timeout -k 10 400 python3 -u -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29744 bench.py --gpus 4 --steps 20 --warmup 5 \
  > $O/bench_n4.log 2>&1; echo "rc=$?"
grep -E "suite \+|WARN|error|rror" $O/bench_n4.log | grep -v amdgpu.ids | head -120
