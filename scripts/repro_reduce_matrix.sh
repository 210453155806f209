#!/bin/bash
# Narrowing a multi-step Reduce parity failure (64 KiB slots, 7 channels): which settings, ranks and
# collectives reproduce it. Each line is one fresh single-process communicator (scripts/repro_case.py).
cd "$GRAFT_REPO_ROOT"
B='"NCCL_AMD_SLOT_BYTES":"65536","NCCL_MAX_CTAS":"7"'
run() { echo "== n=$1 $2 $3"; timeout -k 5 60 python3 -u scripts/repro_case.py "$1" "$2" "$3" 2>&1 | grep -v amdgpu.ids | cut -c1-160; }
run 2 "{$B}" '[["reduce",4,2,1048587,0,1],["reduce",2,0,1048587,0,0]]'
run 3 "{$B}" '[["allreduce",4,2,1048587,0,0],["allreduce",2,0,1048587,0,0]]'
run 3 "{$B}" '[["reduce",7,0,2000001,0,2],["reduce",7,0,2000000,0,1]]'
run 3 "{$B,\"NCCL_AMD_PROTO_FLAGS\":\"3\"}" '[["reduce",2,0,1048587,0,1]]'
run 3 "{$B,\"NCCL_AMD_PROTO_FLAGS\":\"4\"}" '[["reduce",2,0,1048587,0,1]]'
run 3 "{$B,\"NCCL_AMD_FORCE_ELEMENTWISE\":\"1\"}" '[["reduce",2,0,1048587,0,1]]'
run 3 "{$B}" '[["reduce",2,0,1048576,0,1],["reduce",2,0,1048600,0,1]]'
