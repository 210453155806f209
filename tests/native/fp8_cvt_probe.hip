// fp8_cvt_probe — do gfx950's fp8 conversion instructions reproduce the engine's fp8 arithmetic bit for bit?
// Software reference: numerics.h fp8ToF32 / f32ToFp8Sat (checked exhaustively against the oracle on the host,
// tests/test_numerics.py; the reference's __NV_SATFINITE conversion of the half result, reduce_kernel.h:461-487).
// Hardware path (numerics.h fp8ToF32Hw / f32ToFp8SatHw, what the kernels run with NCCL_AMD_HW_FP8=1):
// v_cvt_f32_fp8 / _bf8 and v_cvt_pk_fp8_f32 / _bf8_f32 after a clamp to +-max finite, NaN in software.
// Checks every code (decode) and every half value (encode: the engine rounds to half first). Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../nccl_amd/csrc/numerics.h"

using namespace ncclamd;
typedef float v2f __attribute__((ext_vector_type(2)));

template <bool E5M2>
__device__ inline float hwDecode(uint8_t c) { return fp8ToF32Hw<E5M2>(c); }

template <bool E5M2>
__device__ inline uint8_t hwEncode(float f) { return f32ToFp8SatHw<E5M2>(f); }

// the raw instructions, without the NaN handling (reported: how the hardware treats NaN)
template <bool E5M2>
__device__ inline uint8_t rawEncode(float f) {
  const float mx = E5M2 ? 57344.0f : 448.0f;
  float x = f;
  if (!(x != x)) x = __builtin_fminf(__builtin_fmaxf(x, -mx), mx);
  int r = E5M2 ? __builtin_amdgcn_cvt_pk_bf8_f32(x, x, 0, false) : __builtin_amdgcn_cvt_pk_fp8_f32(x, x, 0, false);
  return (uint8_t)(r & 0xff);
}

template <bool E5M2>
__global__ void probe(unsigned* bad, unsigned* first) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 256) {  // decode: bit-exact, NaN compared as NaN
    float s = fp8ToF32<E5M2>((uint8_t)i), h = hwDecode<E5M2>((uint8_t)i);
    bool same = (s != s) ? (h != h) && (__builtin_bit_cast(uint32_t, s) >> 31) == (__builtin_bit_cast(uint32_t, h) >> 31)
                         : __builtin_bit_cast(uint32_t, s) == __builtin_bit_cast(uint32_t, h);
    if (!same && atomicAdd(&bad[0], 1u) == 0) first[0] = i;
  }
  if (i < 65536) {  // encode every half value
    float f = halfToF32((uint16_t)i);
    uint8_t s = f32ToFp8Sat<E5M2>(f), h = hwEncode<E5M2>(f);
    if (s != h && atomicAdd(&bad[1], 1u) == 0) first[1] = i | ((unsigned)s << 16) | ((unsigned)h << 24);
    if (s != rawEncode<E5M2>(f)) atomicAdd(&bad[2], 1u);  // raw instruction, NaN included
  }
}

int main() {
  unsigned *bad, *first, hb[2][3], hf[2][2];
  if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 16) != hipSuccess) return 1;
  for (int e = 0; e < 2; e++) {
    (void)hipMemset(bad, 0, 16);
    (void)hipMemset(first, 0, 16);
    if (e) hipLaunchKernelGGL(probe<true>, dim3(256), dim3(256), 0, 0, bad, first);
    else hipLaunchKernelGGL(probe<false>, dim3(256), dim3(256), 0, 0, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipMemcpy(hb[e], bad, 12, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf[e], first, 8, hipMemcpyDeviceToHost);
  }
  printf("{\"e4m3_decode_mismatch\": %u, \"e4m3_encode_mismatch\": %u, \"e4m3_raw_encode_mismatch\": %u, "
         "\"e4m3_first\": [%u, %u], \"e5m2_decode_mismatch\": %u, \"e5m2_encode_mismatch\": %u, "
         "\"e5m2_raw_encode_mismatch\": %u, \"e5m2_first\": [%u, %u]}\n",
         hb[0][0], hb[0][1], hb[0][2], hf[0][0], hf[0][1], hb[1][0], hb[1][1], hb[1][2], hf[1][0], hf[1][1]);
  return 0;
}
