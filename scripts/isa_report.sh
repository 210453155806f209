#!/bin/bash
# Packed-arithmetic evidence: disassemble the fp16 / bf16 collective kernels (hipcc --save-temps) and count
# the fold's arithmetic instructions per kernel (sum, prod, premulsum: OP 0 / 1 / 3; COLL 0 = AllReduce).
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
F="-O3 -fPIC -std=c++17 -ffp-contract=off -fvisibility=hidden -Iinclude --offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics"
for k in f16 bf16; do /opt/rocm/bin/hipcc $F --save-temps=obj -c nccl_amd/csrc/kern_$k.hip -o $T/kern_$k.o 2>/dev/null; done
for op in 0 1 3; do
  python3 scripts/isa_count.py $T/kern_f16-hip-amdgcn-amd-amdhsa-gfx950.s "_ZN7ncclamd10collKernelINS_6half_tELi${op}ELi0EEEvNS_8CollArgsE:" "\b(v_pk_\w+|v_\w+_f16\w*|v_cvt_f16\w*|v_cvt_f32_f16\w*|v_fma_mix\w*)\b"
  python3 scripts/isa_count.py $T/kern_bf16-hip-amdgcn-amd-amdhsa-gfx950.s "_ZN7ncclamd10collKernelINS_6bf16_tELi${op}ELi0EEEvNS_8CollArgsE:" "\b(v_pk_\w+|v_cvt_pk\w+|v_mul_f32\w*|v_add_f32\w*)\b"
done
rm -rf $T
