// fp8_f16_probe — gfx950's packed fp8 <-> f16 conversions (v_cvt_scalef32_pk_f16_fp8 / _bf8 decode two codes to
// two halves, v_cvt_scalef32_pk_fp8_f16 / _bf8_f16 encode two halves; scale 1.0) against the engine's software
// conversions (numerics.h fp8ToF32 / f32ToFp8Sat, host-checked against the oracle, tests/test_numerics.py), for
// every code (decode) and every half value (encode, with a NaN-propagating clamp to +-max finite first, the
// reference's __NV_SATFINITE, and raw). Reports mismatches and what the raw instructions do with NaN and with
// out-of-range halves. One JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../nccl_amd/csrc/numerics.h"

using namespace ncclamd;
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));

template <bool E5M2>
__device__ inline h2 dec2(uint32_t w, bool hi) {
  return hi ? (E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w, 1.0f, true) : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, true))
            : (E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w, 1.0f, false) : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, false));
}
template <bool E5M2>
__device__ inline uint32_t enc2(h2 v) {
  const s2 old = {0, 0};
  const s2 r = E5M2 ? __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(old, v, 1.0f, false) : __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(old, v, 1.0f, false);
  return (uint32_t)__builtin_bit_cast(uint32_t, r) & 0xffffu;
}

// stats: 0 decode value mismatches (NaN = NaN, any sign), 1 decode NaN-sign mismatches, 2 clamped-encode
// mismatches (non-NaN inputs), 3 raw-encode mismatches (non-NaN inputs), 4 NaN-input encode results that keep the
// input's sign (0x7f / 0xff pattern as software), 5 NaN inputs seen
template <bool E5M2>
__global__ void probe(unsigned* st, unsigned* first, unsigned* nanCodes) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 256) {
    const uint32_t w = i | (i << 8) | (i << 16) | (i << 24);
    const h2 lo = dec2<E5M2>(w, false), hi = dec2<E5M2>(w, true);
    const float s = fp8ToF32<E5M2>((uint8_t)i);
    const _Float16 got[4] = {lo.x, lo.y, hi.x, hi.y};
    for (int k = 0; k < 4; k++) {
      const float h = (float)got[k];
      const bool sn = s != s, hn = h != h;
      if (sn != hn || (!sn && __builtin_bit_cast(uint32_t, s) != __builtin_bit_cast(uint32_t, h))) {
        if (atomicAdd(&st[0], 1u) == 0) first[0] = i | ((unsigned)__builtin_bit_cast(uint16_t, got[k]) << 16);
      } else if (sn && ((__builtin_bit_cast(uint32_t, s) >> 31) != (__builtin_bit_cast(uint16_t, got[k]) >> 15))) {
        atomicAdd(&st[1], 1u);
      }
    }
  }
  if (i < 65536) {
    const uint16_t hb = (uint16_t)i;
    const _Float16 hv = __builtin_bit_cast(_Float16, hb);
    const float f = (float)hv;
    const uint8_t want = f32ToFp8Sat<E5M2>(f);
    const _Float16 mx = (_Float16)(E5M2 ? 57344.0f : 448.0f);
    const h2 v = {hv, hv}, bound = {mx, mx};
    const h2 c = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, -bound), bound);
    const uint32_t gc = enc2<E5M2>(c), gr = enc2<E5M2>(v);
    if (f != f) {
      atomicAdd(&st[5], 1u);
      if ((gc & 0xff) == want && ((gc >> 8) & 0xff) == want) atomicAdd(&st[4], 1u);
      nanCodes[(hb >> 15) * 2] = gc & 0xff;        // last seen NaN encode per input sign (clamped path)
      nanCodes[(hb >> 15) * 2 + 1] = gr & 0xff;    // raw path
    } else {
      if ((gc & 0xff) != want || ((gc >> 8) & 0xff) != want) {
        if (atomicAdd(&st[2], 1u) == 0) first[1] = i | (gc << 16);
      }
      if ((gr & 0xff) != want && atomicAdd(&st[3], 1u) == 0) first[2] = i | (gr << 16);
    }
  }
}

int main() {
  unsigned *st, *first, *nc, hs[2][6], hf[2][3], hn[2][4];
  if (hipMalloc(&st, 64) != hipSuccess || hipMalloc(&first, 64) != hipSuccess || hipMalloc(&nc, 64) != hipSuccess) return 1;
  for (int e = 0; e < 2; e++) {
    (void)hipMemset(st, 0, 64);
    (void)hipMemset(first, 0, 64);
    (void)hipMemset(nc, 0, 64);
    if (e) hipLaunchKernelGGL(probe<true>, dim3(256), dim3(256), 0, 0, st, first, nc);
    else hipLaunchKernelGGL(probe<false>, dim3(256), dim3(256), 0, 0, st, first, nc);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipMemcpy(hs[e], st, 24, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf[e], first, 12, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hn[e], nc, 16, hipMemcpyDeviceToHost);
  }
  printf("{");
  for (int e = 0; e < 2; e++) {
    const char* f = e ? "e5m2" : "e4m3";
    printf("%s\"%s_decode_mismatch\": %u, \"%s_decode_nan_sign_mismatch\": %u, \"%s_encode_clamped_mismatch\": %u, "
           "\"%s_encode_raw_mismatch\": %u, \"%s_nan_encode_as_software\": %u, \"%s_nan_inputs\": %u, "
           "\"%s_first\": [%u, %u, %u], \"%s_nan_codes_pos_clamped_raw_neg_clamped_raw\": [%u, %u, %u, %u]",
           e ? ", " : "", f, hs[e][0], f, hs[e][1], f, hs[e][2], f, hs[e][3], f, hs[e][4], f, hs[e][5], f, hf[e][0],
           hf[e][1], hf[e][2], f, hn[e][0], hn[e][1], hn[e][2], hn[e][3]);
  }
  printf("}\n");
  return 0;
}
