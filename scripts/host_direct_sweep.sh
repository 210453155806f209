#!/bin/bash
# The host-staged bucket with the collective's kernel on the pinned host buffers (host_pipe_probe.py direct): the
# one-rank copy kernel's grid cap and variant (NCCL_AMD_COPY_GRID / NCCL_AMD_COPY_VARIANT) swept, one JSON line each.
set -e
out=gpurun_out/host_direct
mkdir -p $out
: > $out/sweep.txt
# configurations: the arguments (each "VAR=value[ VAR=value]" or "" for the defaults), else the round-6 sweep
if [ $# -gt 0 ]; then cfgs=("$@"); else
  cfgs=("" "NCCL_AMD_COPY_GRID=256" "NCCL_AMD_COPY_GRID=512" "NCCL_AMD_COPY_GRID=1024" "NCCL_AMD_COPY_GRID=2048"
        "NCCL_AMD_COPY_VARIANT=1" "NCCL_AMD_COPY_VARIANT=3" "NCCL_AMD_COPY_VARIANT=12" "NCCL_AMD_COPY_VARIANT=10"); fi
for cfg in "${cfgs[@]}"; do
  echo -n "${cfg:-default} " >> $out/sweep.txt
  env $cfg HOST_PIPE_CHUNKS= timeout -k 10 90 python -u scripts/host_pipe_probe.py >> $out/sweep.txt 2>>$out/err.txt
done
cat $out/sweep.txt
