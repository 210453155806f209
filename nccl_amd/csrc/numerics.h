// numerics.h — element types and reduction functors of the MI355X kernels.
//
// Semantics follow the reference functors (src/device/reduce_kernel.h):
//   Sum/Prod on integers wrap mod 2^k; signed integers use the unsigned kernels (generate.py:138-146).
//   MinMax on integers: (a^m) < (b^m) ? a : b with the xormask m from hostToDevRedOp
//     (enqueue.cc:2517-2526; reduce_kernel.h:349-356).
//   MinMax on floats: fminf/fmaxf, NaN-ignoring (reduce_kernel.h:409-410, __hmin/__hmax :428-459),
//     with -0 ordered below +0 (see minOrdered).
//   fp16/bf16 Sum/Prod: one IEEE operation rounded RNE to the storage type after every hop
//     (== __hadd/__hmul: an fp32 add/mul of two 11- or 8-bit-significand values rounded once to T is
//     the correctly rounded result).
//   fp8 (OCP e4m3fn / e5m2): computed in half, then converted back with saturation to the largest
//     finite value (reduce_kernel.h:461-487; __NV_SATFINITE).
//   PreMulSum: preOp x*s rounded to T, then Sum (reduce_kernel.h:586-712). SumPostDiv (integer avg):
//     Sum, then divide the wrapped sum by n, sign-magnitude (reduce_kernel.h:936-966).
// The kernels are built with -ffp-contract=off so x*s + acc is never fused into one FMA.
//
// All helpers are __host__ __device__ so tests/ can check them exhaustively on the host against the
// independent C oracle (oracle/nccl_oracle.c).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ncclamd {

struct half_t { uint16_t x; };
struct bf16_t { uint16_t x; };
struct e4m3_t { uint8_t x; };
struct e5m2_t { uint8_t x; };

__host__ __device__ inline float u32AsF32(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ inline uint32_t f32AsU32(float f) { return __builtin_bit_cast(uint32_t, f); }

// ---- fp16 ----
__host__ __device__ inline float halfToF32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__host__ __device__ inline uint16_t f32ToHalf(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// ---- bf16: RNE with NaN kept NaN (v_cvt_pk_bf16_f32 on gfx950) ----
__host__ __device__ inline float bf16ToF32(uint16_t b) { return u32AsF32((uint32_t)b << 16); }
__host__ __device__ inline uint16_t f32ToBf16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(uint16_t, (__bf16)f);
#else
  uint32_t u = f32AsU32(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
#endif
}

// ---- fp8 (OCP). Decode is exact; encode rounds RNE and saturates to max finite. ----
template <bool E5M2>
__host__ __device__ inline float fp8ToF32(uint8_t v) {
  uint32_t sign = (uint32_t)(v & 0x80) << 24;
  if (E5M2) {
    uint32_t e = (v >> 2) & 0x1f, m = v & 3;
    if (e == 31) return u32AsF32(sign | 0x7f800000u | (m ? 0x400000u : 0u));
    if (e == 0) return u32AsF32(sign | f32AsU32((float)m * (1.0f / 65536.0f)));
    return u32AsF32(sign | ((e + 112) << 23) | (m << 21));
  } else {
    uint32_t e = (v >> 3) & 0xf, m = v & 7;
    if (e == 15 && m == 7) return u32AsF32(sign | 0x7fc00000u);
    if (e == 0) return u32AsF32(sign | f32AsU32((float)m * (1.0f / 512.0f)));
    return u32AsF32(sign | ((e + 120) << 23) | (m << 20));
  }
}

template <bool E5M2>
__host__ __device__ inline uint8_t f32ToFp8Sat(float f) {
  uint32_t u = f32AsU32(f);
  uint8_t sign = (uint8_t)((u >> 24) & 0x80);
  uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return sign | 0x7f;  // NaN
  constexpr uint32_t kMax = E5M2 ? 0x47600000u : 0x43e00000u;     // 57344 / 448
  constexpr uint32_t kMinNorm = E5M2 ? 0x38800000u : 0x3c800000u; // 2^-14 / 2^-6
  constexpr uint8_t kMaxCode = E5M2 ? 0x7b : 0x7e;
  constexpr int kMan = E5M2 ? 2 : 3;
  constexpr int kBiasAdj = E5M2 ? 112 : 120;  // 127 - bias
  if (a >= kMax) return sign | kMaxCode;
  if (a < kMinNorm) {
    // subnormal quantum 2^-16 / 2^-9: scale exactly, round to nearest even integer
    float q = u32AsF32(a) * (E5M2 ? 65536.0f : 512.0f);
    uint32_t qi = (uint32_t)q;
    float frac = q - (float)qi;
    if (frac > 0.5f || (frac == 0.5f && (qi & 1))) qi++;
    return sign | (uint8_t)qi;  // qi == 2^kMan becomes the smallest normal code
  }
  uint32_t e = (a >> 23) - kBiasAdj;
  uint32_t man = a & 0x7fffffu;
  uint32_t code = (e << kMan) | (man >> (23 - kMan));
  uint32_t rem = man & ((1u << (23 - kMan)) - 1);
  uint32_t halfway = 1u << (22 - kMan);
  if (rem > halfway || (rem == halfway && (code & 1))) code++;
  if (code > kMaxCode) code = kMaxCode;
  return sign | (uint8_t)code;
}

// ---- fp8 through gfx950's convert instructions (device only) ----
// v_cvt_f32_fp8 / _bf8 decode one OCP code exactly; v_cvt_pk_fp8_f32 / _bf8_f32 encode with round to nearest
// even. tests/native/fp8_cvt_probe (GPU test tests/test_gpu_numerics.py) checks these two functions against the
// software ones above for every code and every half value: they differ only in NaN sign handling (the hardware
// decodes 0x7f as a negative NaN and encodes every NaN as 0xff), so NaN takes the software result; saturation
// (__NV_SATFINITE) is a clamp to +-max finite before the round, exact because the input is a half value (fromF
// rounds to half first). Each replaces ~20 integer ops of the software conversion by one instruction.
#ifndef NCCL_AMD_HW_FP8
#define NCCL_AMD_HW_FP8 1
#endif
#if defined(__HIP__)  // HIP compilations only (the host-only numerics test build is plain C++)
template <bool E5M2>
__device__ inline float fp8ToF32Hw(uint8_t v) {
  const float f = E5M2 ? __builtin_amdgcn_cvt_f32_bf8((int)v, 0) : __builtin_amdgcn_cvt_f32_fp8((int)v, 0);
  const bool nan = E5M2 ? ((v & 0x7c) == 0x7c && (v & 3) != 0) : ((v & 0x7f) == 0x7f);
  return nan ? u32AsF32(((uint32_t)(v & 0x80) << 24) | 0x7fc00000u) : f;
}
template <bool E5M2>
__device__ inline uint8_t f32ToFp8SatHw(float f) {  // f must be a half value
  if (f != f) return (uint8_t)(((f32AsU32(f) >> 24) & 0x80) | 0x7f);
  const float mx = E5M2 ? 57344.0f : 448.0f;
  const float x = __builtin_fminf(__builtin_fmaxf(f, -mx), mx);
  const int r = E5M2 ? __builtin_amdgcn_cvt_pk_bf8_f32(x, x, 0, false) : __builtin_amdgcn_cvt_pk_fp8_f32(x, x, 0, false);
  return (uint8_t)(r & 0xff);
}
#endif

// ---- min/max with a defined signed-zero order ----
// The reference uses fminf/fmaxf (reduce_kernel.h:409-410) and __hmin/__hmax: NaN-ignoring, but the
// result for (+0, -0) is implementation-defined in C. Here -0 orders below +0 (IEEE 754-2019
// minimumNumber/maximumNumber), identically on host and device, so results never depend on the
// instruction the compiler picks.
template <typename F>
__host__ __device__ inline F minOrdered(F a, F b) {
  if (a != a) return b;
  if (b != b) return a;
  if (a < b) return a;
  if (b < a) return b;
  return __builtin_signbit(a) ? a : b;
}
template <typename F>
__host__ __device__ inline F maxOrdered(F a, F b) {
  if (a != a) return b;
  if (b != b) return a;
  if (a > b) return a;
  if (b > a) return b;
  return __builtin_signbit(a) ? b : a;
}

// ---- per-type traits: load as f32 ("compute" value) and store back with the type's rounding ----
template <typename T> struct Traits;
template <> struct Traits<uint8_t>  { static constexpr bool isFloat = false; };
template <> struct Traits<uint16_t> { static constexpr bool isFloat = false; };
template <> struct Traits<uint32_t> { static constexpr bool isFloat = false; };
template <> struct Traits<uint64_t> { static constexpr bool isFloat = false; };
template <> struct Traits<float>    { static constexpr bool isFloat = true; };
template <> struct Traits<double>   { static constexpr bool isFloat = true; };
template <> struct Traits<half_t> {
  static constexpr bool isFloat = true;
  __host__ __device__ static float toF(half_t v) { return halfToF32(v.x); }
  __host__ __device__ static half_t fromF(float f) { return half_t{f32ToHalf(f)}; }
};
template <> struct Traits<bf16_t> {
  static constexpr bool isFloat = true;
  __host__ __device__ static float toF(bf16_t v) { return bf16ToF32(v.x); }
  __host__ __device__ static bf16_t fromF(float f) { return bf16_t{f32ToBf16(f)}; }
};
template <bool E5M2>
__host__ __device__ inline float fp8Decode(uint8_t v) {
#if defined(__HIP_DEVICE_COMPILE__) && NCCL_AMD_HW_FP8
  return fp8ToF32Hw<E5M2>(v);
#else
  return fp8ToF32<E5M2>(v);
#endif
}
// the reference's fp8 ops run on __half and convert back with saturation: round to half first
template <bool E5M2>
__host__ __device__ inline uint8_t fp8Encode(float f) {
#if defined(__HIP_DEVICE_COMPILE__) && NCCL_AMD_HW_FP8
  return f32ToFp8SatHw<E5M2>(halfToF32(f32ToHalf(f)));
#else
  return f32ToFp8Sat<E5M2>(halfToF32(f32ToHalf(f)));
#endif
}
template <> struct Traits<e4m3_t> {
  static constexpr bool isFloat = true;
  __host__ __device__ static float toF(e4m3_t v) { return fp8Decode<false>(v.x); }
  __host__ __device__ static e4m3_t fromF(float f) { return e4m3_t{fp8Encode<false>(f)}; }
};
template <> struct Traits<e5m2_t> {
  static constexpr bool isFloat = true;
  __host__ __device__ static float toF(e5m2_t v) { return fp8Decode<true>(v.x); }
  __host__ __device__ static e5m2_t fromF(float f) { return e5m2_t{fp8Encode<true>(f)}; }
};

// ---- functors: pre(x), red(preLocal, acc), post(acc) ----
template <typename T, int OP> struct Red;

// integers (unsigned storage)
template <typename T, int OP>
struct RedInt {
  T arg;  // xormask (MinMax) / scalar (PreMulSum)
  uint32_t divisor;
  bool isSigned;
  __host__ __device__ explicit RedInt(uint64_t a) : arg((T)a), divisor((uint32_t)(a >> 1)), isSigned(a & 1) {}
  __host__ __device__ T pre(T x) const { return OP == 3 ? (T)(x * arg) : x; }
  __host__ __device__ T red(T a, T b) const {
    if (OP == 1) return (T)(a * b);
    if (OP == 2) return (T)(a ^ arg) < (T)(b ^ arg) ? a : b;
    return (T)(a + b);
  }
  __host__ __device__ T post(T x) const {
    if (OP != 4) return x;
    const T signBit = (T)((T)1 << (sizeof(T) * 8 - 1));
    bool neg = isSigned && (x & signBit);
    T xabs = neg ? (T)(0 - x) : x;
    T q = (T)(xabs / (T)divisor);
    return neg ? (T)(0 - q) : q;
  }
};
template <int OP> struct Red<uint8_t, OP> : RedInt<uint8_t, OP> { using RedInt<uint8_t, OP>::RedInt; };
template <int OP> struct Red<uint16_t, OP> : RedInt<uint16_t, OP> { using RedInt<uint16_t, OP>::RedInt; };
template <int OP> struct Red<uint32_t, OP> : RedInt<uint32_t, OP> { using RedInt<uint32_t, OP>::RedInt; };
template <int OP> struct Red<uint64_t, OP> : RedInt<uint64_t, OP> { using RedInt<uint64_t, OP>::RedInt; };

template <int OP> struct Red<float, OP> {
  float s;
  bool isMin;
  __host__ __device__ explicit Red(uint64_t a) : s(u32AsF32((uint32_t)a)), isMin((a & 1) == 0) {}
  __host__ __device__ float pre(float x) const { return OP == 3 ? x * s : x; }
  __host__ __device__ float red(float a, float b) const {
    if (OP == 1) return a * b;
    if (OP == 2) return isMin ? minOrdered(a, b) : maxOrdered(a, b);
    return a + b;
  }
  __host__ __device__ float post(float x) const { return x; }
};
template <int OP> struct Red<double, OP> {
  double s;
  bool isMin;
  __host__ __device__ explicit Red(uint64_t a) : s(__builtin_bit_cast(double, a)), isMin((a & 1) == 0) {}
  __host__ __device__ double pre(double x) const { return OP == 3 ? x * s : x; }
  __host__ __device__ double red(double a, double b) const {
    if (OP == 1) return a * b;
    if (OP == 2) return isMin ? minOrdered(a, b) : maxOrdered(a, b);
    return a + b;
  }
  __host__ __device__ double post(double x) const { return x; }
};

// Keep an f32 result opaque to the optimiser before it is rounded to a narrower type: at -O3 the
// backend folds fptrunc(fmul(x, y)) into v_fma_mixlo_f16(x, y, +0.0), which turns (-0)*y into +0
// (found by the fp8 avg parity test). The empty asm forces a plain v_mul_f32 + v_cvt.
__host__ __device__ inline float opaqueF(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}

// small floats: compute in f32, round to T after every operation
template <typename T, int OP>
struct RedSmall {
  float s;
  bool isMin;
  __host__ __device__ explicit RedSmall(uint64_t a) {
    T sv;
    __builtin_memcpy(&sv, &a, sizeof(T));
    s = Traits<T>::toF(sv);
    isMin = (a & 1) == 0;
  }
  __host__ __device__ T pre(T x) const { return OP == 3 ? Traits<T>::fromF(opaqueF(Traits<T>::toF(x) * s)) : x; }
  __host__ __device__ T red(T a, T b) const {
    float x = Traits<T>::toF(a), y = Traits<T>::toF(b), r;
    if (OP == 1) r = opaqueF(x * y);
    else if (OP == 2) r = isMin ? minOrdered(x, y) : maxOrdered(x, y);
    else r = x + y;
    return Traits<T>::fromF(r);
  }
  __host__ __device__ T post(T x) const { return x; }
};
// fp16: native half arithmetic (reference __hadd/__hmul/__hadd2, reduce_kernel.h:411-459). One IEEE fp16
// add or multiply, rounded RNE, is exactly the oracle's f32 operation rounded once to half (the exact sum of
// two 11-bit significands fits f32 whenever it can matter; their product always does), so results are
// bit-identical — and a fold over 16-byte packs compiles to v_pk_add_f16 / v_pk_mul_f16, two lanes per
// instruction. Min/max keep the f32 path with the defined signed-zero order (minOrdered).
template <int OP>
struct Red<half_t, OP> {
  _Float16 s;
  bool isMin;
  __host__ __device__ static _Float16 h(half_t v) { return __builtin_bit_cast(_Float16, v.x); }
  __host__ __device__ static half_t w(_Float16 v) { return half_t{__builtin_bit_cast(uint16_t, v)}; }
  __host__ __device__ explicit Red(uint64_t a) : s(__builtin_bit_cast(_Float16, (uint16_t)a)), isMin((a & 1) == 0) {}
  __host__ __device__ half_t pre(half_t x) const { return OP == 3 ? w(h(x) * s) : x; }
  __host__ __device__ half_t red(half_t a, half_t b) const {
    if (OP == 1) return w(h(a) * h(b));
    if (OP == 2) {
      float x = halfToF32(a.x), y = halfToF32(b.x);
      return half_t{f32ToHalf(isMin ? minOrdered(x, y) : maxOrdered(x, y))};
    }
    return w(h(a) + h(b));
  }
  __host__ __device__ half_t post(half_t x) const { return x; }
};
// bf16: f32 arithmetic on the widened values, then one RNE rounding (gfx950 has no bf16 VALU add; the
// widening is a shift / mask, the f32 pairs go to v_pk_add_f32 / v_pk_mul_f32 and the rounding of two
// results to v_cvt_pk_bf16_f32). No opaque barrier is needed here: there is no mixed-precision bf16 FMA
// the backend could fold a rounded product into (that hazard is fp16 / fp8 only, see opaqueF).
template <int OP>
struct Red<bf16_t, OP> {
  float s;
  bool isMin;
  __host__ __device__ explicit Red(uint64_t a) : s(bf16ToF32((uint16_t)a)), isMin((a & 1) == 0) {}
  __host__ __device__ bf16_t pre(bf16_t x) const { return OP == 3 ? bf16_t{f32ToBf16(bf16ToF32(x.x) * s)} : x; }
  __host__ __device__ bf16_t red(bf16_t a, bf16_t b) const {
    float x = bf16ToF32(a.x), y = bf16ToF32(b.x), r;
    if (OP == 1) r = x * y;
    else if (OP == 2) r = isMin ? minOrdered(x, y) : maxOrdered(x, y);
    else r = x + y;
    return bf16_t{f32ToBf16(r)};
  }
  __host__ __device__ bf16_t post(bf16_t x) const { return x; }
};
template <int OP> struct Red<e4m3_t, OP> : RedSmall<e4m3_t, OP> { using RedSmall<e4m3_t, OP>::RedSmall; };
template <int OP> struct Red<e5m2_t, OP> : RedSmall<e5m2_t, OP> { using RedSmall<e5m2_t, OP>::RedSmall; };

// ---- fp8 packs: four codes per dword through the paired convert instructions (device only) ----
// The staged / zero-copy fold keeps an fp8 accumulator as the f32 VALUES of its codes between sources and
// rounds each hop with fp8RoundF (the value fromF would store: RNE to half, satfinite, RNE to fp8), encoding
// only once at the end: per element one half round trip, a clamp and half a paired encode + decode per hop,
// instead of a full decode + encode per hop. Bit-identical to Red<e4m3_t / e5m2_t, OP> per element (the
// decode / encode instructions equal the software conversions on every code and every half value,
// tests/native/fp8_cvt_probe; tests/test_gpu_numerics.py runs every code pair through both paths).
template <typename T> struct IsFp8 { static constexpr bool value = false; };
template <> struct IsFp8<e4m3_t> { static constexpr bool value = true; static constexpr bool e5m2 = false; };
template <> struct IsFp8<e5m2_t> { static constexpr bool value = true; static constexpr bool e5m2 = true; };

#if defined(__HIP__)
typedef float fp8v2f __attribute__((ext_vector_type(2)));
__device__ inline float withSignOf(float x, uint32_t s) {  // x's magnitude, bit 31 of s: one v_bfi_b32
  // (written as and / and / or, the backend emits three instructions; a VALU-only asm has no hazards)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x7fffffffu), "v"(f32AsU32(x)), "v"(s));  // gfx9 VOP3: no literal
  return u32AsF32(r);
}
// four codes -> four values; NaN codes keep their own sign (the instruction makes every NaN negative)
template <bool E5M2>
__device__ inline void fp8Decode4(uint32_t w, float* f) {
  const fp8v2f lo = E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8((int)w, false) : __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
  const fp8v2f hi = E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8((int)w, true) : __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  f[0] = withSignOf(lo.x, w << 24);
  f[1] = withSignOf(lo.y, w << 16);
  f[2] = withSignOf(hi.x, w << 8);
  f[3] = withSignOf(hi.y, w);
}
// the values fromF would store for a and b: RNE to half, then satfinite RNE to fp8 (paired encode + decode);
// NaN stays NaN with its sign
template <bool E5M2>
__device__ inline void fp8RoundF(float& a, float& b) {
  const float mx = E5M2 ? 57344.0f : 448.0f;
  const float ha = halfToF32(f32ToHalf(a)), hb = halfToF32(f32ToHalf(b));
  const float ca = __builtin_fminf(__builtin_fmaxf(ha, -mx), mx), cb = __builtin_fminf(__builtin_fmaxf(hb, -mx), mx);
  // the high word of the paired encode is never read: any register serves as its "old" operand (no v_mov)
  const int old = (int)f32AsU32(ca);
  const int w = E5M2 ? __builtin_amdgcn_cvt_pk_bf8_f32(ca, cb, old, false) : __builtin_amdgcn_cvt_pk_fp8_f32(ca, cb, old, false);
  const fp8v2f d = E5M2 ? __builtin_amdgcn_cvt_pk_f32_bf8(w, false) : __builtin_amdgcn_cvt_pk_f32_fp8(w, false);
  a = ha != ha ? ha : d.x;
  b = hb != hb ? hb : d.y;
}
// ---- fp8 packs as packed halves (gfx950 v_cvt_scalef32_pk_f16_fp8 / _pk_fp8_f16, scale 1.0) ----
// The reference computes every fp8 operation in half and converts back with saturation (reduce_kernel.h:461-487):
// v_pk_add_f16 / v_pk_mul_f16 ARE __hadd / __hmul on two lanes, v_pk_maximum3_f16 / v_pk_minimum3_f16 clamp to
// +-max finite (__NV_SATFINITE), and the packed converts move two codes per instruction. Probed on the MI355X
// against the software conversions for every code and every half value (tests/native/fp8_f16_probe,
// profiles/r03_fp8_f16_probe.json): decode exact, clamped encode exact, only NaN differs (every NaN decodes
// negative; NaN encodes 0xff / 0xfe). The packed fold therefore runs only on packs with no NaN / Inf code in any
// source (fp8Special): finite fp8 inputs never create NaN or Inf under satfinite, and a pack that holds one is
// recomputed by the f32 path above.
typedef _Float16 fp8h2 __attribute__((ext_vector_type(2)));
typedef short fp8s2 __attribute__((ext_vector_type(2)));
// codes 0, 1 (hi = false) or 2, 3 (hi = true) of w -> their values as two halves
template <bool E5M2>
__device__ inline fp8h2 fp8DecodeH2(uint32_t w, bool hi) {
  if (hi) return E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w, 1.0f, true) : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, true);
  return E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w, 1.0f, false) : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, false);
}
// nonzero when a byte of w is a NaN code (e4m3 S.1111.111) or a NaN / Inf code (e5m2 S.11111.xx)
template <bool E5M2>
__device__ inline uint32_t fp8Special(uint32_t w) {
  return ((w & 0x7f7f7f7fu) + (E5M2 ? 0x04040404u : 0x01010101u)) & 0x80808080u;
}
// two finite half results -> the fp8 values fromF would store (satfinite clamp, RNE encode, decode)
template <bool E5M2>
__device__ inline fp8h2 fp8RoundH2(fp8h2 v) {
  const _Float16 m = (_Float16)(E5M2 ? 57344.0f : 448.0f);
  const fp8h2 hiB = {m, m}, loB = {-m, -m};
  v = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, loB), hiB);
  const fp8s2 old = __builtin_bit_cast(fp8s2, v);  // the high word of the encode is never read
  const fp8s2 c = E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(old, v, 1.0f, false)
                       : __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(old, v, 1.0f, false);
  return fp8DecodeH2<E5M2>(__builtin_bit_cast(uint32_t, c), false);
}
// four finite fp8 values (two halves each in a, b) -> four codes (exact: no rounding happens)
template <bool E5M2>
__device__ inline uint32_t fp8EncodeH2x2(fp8h2 a, fp8h2 b) {
  fp8s2 w = __builtin_bit_cast(fp8s2, a);
  w = E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(w, a, 1.0f, false) : __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(w, a, 1.0f, false);
  w = E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(w, b, 1.0f, true) : __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(w, b, 1.0f, true);
  return __builtin_bit_cast(uint32_t, w);
}

// four fp8 VALUES (fp8RoundF results or decoded codes: exact, no rounding) -> four codes; NaN -> sign | 0x7f, the
// software encoder's (and the LL path's) NaN
template <bool E5M2>
__device__ inline uint32_t fp8Encode4(const float* f) {
  const int old = (int)f32AsU32(f[0]);  // high word overwritten below
  int w = E5M2 ? __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], old, false) : __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], old, false);
  w = E5M2 ? __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w, true) : __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
  // the instruction encodes every NaN as 0xff (e4m3) / 0xfe (e5m2): a positive NaN clears bit 7 of its byte, and an
  // e5m2 NaN also sets bit 0 (0xfe -> 0xff), so every path stores sign | 0x7f (tests/test_gpu_collectives.py test_single_nan_payloads)
  uint32_t clr = 0, set = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t a = f32AsU32(f[i]) & 0x7fffffffu;
    clr |= f32AsU32(f[i]) - 0x7f800001u < 0x007fffffu ? 0x80u << (8 * i) : 0u;  // +NaN
    if (E5M2) set |= a > 0x7f800000u ? 0x01u << (8 * i) : 0u;                      // any NaN
  }
  return ((uint32_t)w | set) & ~clr;
}
#endif

// ---- 1-byte integer Sum / MinMax on four bytes per dword (SWAR) ----
// Bit-identical to Red<uint8_t, OP>::red on each byte (tests/test_numerics.py checks every byte pair). The fold
// uses it for uint8 / int8 so a 16-byte pack stays four registers instead of sixteen unpacked bytes, which
// lets it keep four packs per thread in flight within the 128-VGPR co-residency budget.
template <int OP> struct Swar8 { static constexpr bool ok = false; };
template <> struct Swar8<0> {  // DEV_SUM: byte-wise add mod 256 (carries masked out of each byte)
  static constexpr bool ok = true;
  __host__ __device__ static uint32_t red(uint32_t a, uint32_t b, uint32_t) {
    return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
  }
};
template <> struct Swar8<2> {  // DEV_MINMAX: (a^m) < (b^m) ? a : b per byte; M = the xormask in every byte
  static constexpr bool ok = true;
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  __host__ __device__ static uint32_t red(uint32_t a, uint32_t b, uint32_t M) {
    const uint32_t x = a ^ M, y = b ^ M;  // unsigned order of x, y = the functor's order of a, b
    const us2 lo = __builtin_elementwise_min(__builtin_bit_cast(us2, x & 0x00ff00ffu),
                                             __builtin_bit_cast(us2, y & 0x00ff00ffu));  // v_pk_min_u16
    const us2 hi = __builtin_elementwise_min(__builtin_bit_cast(us2, (x >> 8) & 0x00ff00ffu),
                                             __builtin_bit_cast(us2, (y >> 8) & 0x00ff00ffu));
    return (__builtin_bit_cast(uint32_t, lo) | (__builtin_bit_cast(uint32_t, hi) << 8)) ^ M;
  }
};

// SumPostDiv on 1-byte integers (integer avg): the fold is the byte-wise Sum (Swar8<0>, the sum wraps mod 256 for
// either signedness) and the post-op divides each byte: magnitude / n, sign restored for signed types
// (reduce_kernel.h:936-966). For a magnitude x <= 255 and a divisor 1 <= d <= 256 the quotient is
// (x * M) >> 16 with M = ceil(2^16 / d) exactly (x * (M d - 2^16) < x d < 2^16), so no division is issued.
// Bit-identical to Red<uint8_t, DEV_SUMPOSTDIV>::post on each byte (tests/test_numerics.py, every byte and d).
__host__ __device__ inline uint32_t swarDivMagic(uint32_t d) { return (65536u + d - 1) / d; }
__host__ __device__ inline uint32_t swarDivBytes(uint32_t w, uint32_t M, bool isSigned) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t x = (w >> (8 * b)) & 0xffu;
    const bool neg = isSigned && (x & 0x80u);
    const uint32_t mag = neg ? ((0u - x) & 0xffu) : x;
    uint32_t q = (mag * M) >> 16;
    if (neg) q = 0u - q;
    r |= (q & 0xffu) << (8 * b);
  }
  return r;
}

}  // namespace ncclamd
