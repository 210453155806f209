#!/bin/bash
cd "$GRAFT_REPO_ROOT"
B='"NCCL_AMD_SLOT_BYTES":"65536","NCCL_MAX_CTAS":"7"'
run() { echo "== n=$1 $2 $3"; timeout -k 5 60 python3 -u scripts/repro_case.py "$1" "$2" "$3" 2>&1 | grep -v amdgpu.ids | cut -c1-200; }
run 2 "{$B}" '[["allreduce",7,0,1048576,0,0],["allreduce",2,0,1048576,0,0],["allreduce",3,0,1048576,0,0],["allreduce",7,1,1048576,0,0],["allreduce",2,0,2000000,0,0],["allreduce",7,0,2097152,0,0]]'
run 2 "{\"NCCL_AMD_SLOT_BYTES\":\"65536\"}" '[["allreduce",2,0,1048576,0,0],["allreduce",2,0,16777216,0,0]]'
run 2 "{\"NCCL_MAX_CTAS\":\"7\"}" '[["allreduce",2,0,1048576,0,0],["allreduce",2,0,16777216,0,0]]'
run 2 "{$B,\"NCCL_AMD_NSLOTS\":\"1\"}" '[["allreduce",2,0,1048576,0,0]]'
