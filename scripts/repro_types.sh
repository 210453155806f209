#!/bin/bash
cd "$GRAFT_REPO_ROOT"
B='{"NCCL_AMD_SLOT_BYTES":"65536","NCCL_MAX_CTAS":"7"}'
timeout -k 5 120 python3 -u scripts/repro_case.py 2 "$B" '[["allreduce",0,0,4194304,0,0],["allreduce",1,0,4194304,0,0],["allreduce",4,0,524288,0,0],["allreduce",5,0,524288,0,0],["allreduce",6,0,2097152,0,0],["allreduce",9,0,2097152,0,0],["allreduce",8,0,524288,0,0],["allreduce",7,0,1048576,0,0],["allreduce",2,2,1048576,0,0],["allreduce",2,1,1048576,0,0],["allreduce",7,2,1048576,0,0],["allreduce",10,0,4194304,0,0]]' 2>&1 | grep -v amdgpu.ids | cut -c1-120
