// Host build of the kernels' numerics (nccl_amd/csrc/numerics.h) for exhaustive CPU checks against
// the independent C oracle (tests/test_numerics.py). Test-only; not part of libnccl.so.
#include "../../nccl_amd/csrc/numerics.h"
using namespace ncclamd;
extern "C" {
uint16_t nx_f32_to_half(float f) { return f32ToHalf(f); }
float nx_half_to_f32(uint16_t h) { return halfToF32(h); }
uint16_t nx_f32_to_bf16(float f) { return f32ToBf16(f); }
float nx_bf16_to_f32(uint16_t h) { return bf16ToF32(h); }
float nx_fp8_to_f32(uint8_t v, int e5m2) { return e5m2 ? fp8ToF32<true>(v) : fp8ToF32<false>(v); }
uint8_t nx_f32_to_fp8(float f, int e5m2) { return e5m2 ? f32ToFp8Sat<true>(f) : f32ToFp8Sat<false>(f); }
// one reduction step on raw storage bits: dtype = ncclDataType_t, op = DevRedOp, arg = redArg
uint64_t nx_red(int dtype, int op, uint64_t arg, uint64_t a, uint64_t b);
uint64_t nx_pre(int dtype, int op, uint64_t arg, uint64_t a);
uint64_t nx_post(int dtype, int op, uint64_t arg, uint64_t a);
uint32_t nx_swar8(int op, uint32_t mask, uint32_t a, uint32_t b);
uint32_t nx_swar_div(uint32_t w, uint32_t d, int isSigned) { return swarDivBytes(w, swarDivMagic(d), isSigned != 0); }
}
uint32_t nx_swar8(int op, uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t M = (mask & 0xff) * 0x01010101u;
  return op == 0 ? Swar8<0>::red(a, b, M) : Swar8<2>::red(a, b, M);
}
template <typename T, int OP> static uint64_t red1(uint64_t arg, uint64_t a, uint64_t b, int which) {
  Red<T, OP> fn(arg);
  T x, y; __builtin_memcpy(&x, &a, sizeof(T)); __builtin_memcpy(&y, &b, sizeof(T));
  T r = which == 0 ? fn.red(x, y) : which == 1 ? fn.pre(x) : fn.post(x);
  uint64_t o = 0; __builtin_memcpy(&o, &r, sizeof(T)); return o;
}
template <typename T> static uint64_t byOp(int op, uint64_t arg, uint64_t a, uint64_t b, int which) {
  switch (op) {
    case 0: return red1<T, 0>(arg, a, b, which);
    case 1: return red1<T, 1>(arg, a, b, which);
    case 2: return red1<T, 2>(arg, a, b, which);
    case 3: return red1<T, 3>(arg, a, b, which);
    default: return red1<T, 4>(arg, a, b, which);
  }
}
static uint64_t dispatch(int dt, int op, uint64_t arg, uint64_t a, uint64_t b, int which) {
  switch (dt) {
    case 0: case 1: return byOp<uint8_t>(op, arg, a, b, which);
    case 2: case 3: return byOp<uint32_t>(op, arg, a, b, which);
    case 4: case 5: return byOp<uint64_t>(op, arg, a, b, which);
    case 6: return op == 4 ? 0 : byOp<half_t>(op, arg, a, b, which);
    case 7: return op == 4 ? 0 : byOp<float>(op, arg, a, b, which);
    case 8: return op == 4 ? 0 : byOp<double>(op, arg, a, b, which);
    case 9: return op == 4 ? 0 : byOp<bf16_t>(op, arg, a, b, which);
    case 10: return op == 4 ? 0 : byOp<e4m3_t>(op, arg, a, b, which);
    default: return op == 4 ? 0 : byOp<e5m2_t>(op, arg, a, b, which);
  }
}
uint64_t nx_red(int dt, int op, uint64_t arg, uint64_t a, uint64_t b) { return dispatch(dt, op, arg, a, b, 0); }
uint64_t nx_pre(int dt, int op, uint64_t arg, uint64_t a) { return dispatch(dt, op, arg, a, 0, 1); }
uint64_t nx_post(int dt, int op, uint64_t arg, uint64_t a) { return dispatch(dt, op, arg, a, 0, 2); }
