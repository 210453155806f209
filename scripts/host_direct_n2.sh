#!/bin/bash
# host_direct_n2.py under channel caps; one JSON line per setting
set -e
out=gpurun_out/host_direct
mkdir -p $out
: > $out/n2.txt
for cfg in "" "NCCL_MAX_CTAS=256" "NCCL_MAX_CTAS=128" "NCCL_MAX_CTAS=64" "NCCL_MAX_CTAS=32" "NCCL_MAX_CTAS=16"; do
  env $cfg timeout -k 10 90 python -u scripts/host_direct_n2.py >> $out/n2.txt 2>>$out/n2_err.txt
done
cat $out/n2.txt
