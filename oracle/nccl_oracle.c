/*
 * nccl_oracle.c — CPU restatement of the reference's reduction semantics. TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X engine. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it (as oracle/_build/liboracle.so). The product library
 * (nccl_amd/lib/libnccl.so) never links or calls it.
 *
 * What it restates (reference = NVIDIA/nccl 2.30.7 at /root/reference; citations are path:line):
 *   - op mapping hostToDevRedOp                         src/enqueue.cc:2479-2583
 *   - reduction functors Sum/Prod/MinMax                 src/device/reduce_kernel.h:41-66, 330-357
 *   - half/bf16 arithmetic (__hadd/__hmul/__hmin/__hmax) src/device/reduce_kernel.h:411-459
 *   - fp8 arithmetic via half                            src/device/reduce_kernel.h:461-487
 *   - PreMulSum pre-op (avg on floats, user premul op)   src/device/reduce_kernel.h:586-712
 *   - SumPostDiv post-op (avg on integers)               src/device/reduce_kernel.h:936-966
 *   - operand order acc = f(preOp(local input), acc)     src/device/common_kernel.h:83-121
 *   - ring fold order: the value owned by ring position c is folded starting at c+1, c+2, ...,
 *     ending with c's own input, rounded to T after every hop:
 *       AllReduce      src/device/all_reduce.h:13-83 (chunk c finalised at ringIx c; one channel,
 *                      one loop iteration: chunkCount = alignUp(divUp(count,n), 16/sizeof(T)), :38);
 *                      at full size on K channels (RING/SIMPLE): oracle_all_reduce_ring_nccl, the
 *                      reference's channel parts and loops (enqueue.cc:576-757, 2070-2097, 2182-2321)
 *       ReduceScatter  src/device/reduce_scatter.h:13-56 (block d finalised at rank d)
 *       Reduce         src/device/reduce.h:13-53 (chain: root+1 sends, root reduces last)
 *     Ring order is the identity permutation (ring index = rank, src/init.cc:791-808 on a full mesh).
 *
 * Pinning: the reference ships no golden vectors (nccl-tests is external, README.md:78-88). The
 * oracle is pinned by the reference's known-answer tests — docs/examples/03_collectives/01_allreduce
 * (c/main.cc:112-168, python/allreduce.py:97-116: every element = n(n-1)/2) and
 * docs/examples/05_symmetric_memory/02_allgather/c/main.cc:160-175 (segment r = r) — plus fixtures
 * produced by an independent numpy restatement (tests/golden/make_golden.py). fp16/bf16/fp8 hop
 * arithmetic follows the published IEEE RNE semantics of cuda_fp16.h/cuda_bf16.h/cuda_fp8.h, which
 * are not vendored in the reference: that boundary is "parity unpinned" (see DESIGN.md).
 *
 * Also here: the OpenMP host element-wise reduction used as bench.py's naive CPU baseline
 *  — same fold order, so it doubles as an oracle for large sizes.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ncclDataType_t values (nccl.h.in:382-395) */
enum { DT_I8 = 0, DT_U8 = 1, DT_I32 = 2, DT_U32 = 3, DT_I64 = 4, DT_U64 = 5, DT_F16 = 6, DT_F32 = 7,
       DT_F64 = 8, DT_BF16 = 9, DT_E4M3 = 10, DT_E5M2 = 11, DT_NUM = 12 };
/* ncclRedOp_t values (nccl.h.in:364-372) */
enum { OP_SUM = 0, OP_PROD = 1, OP_MAX = 2, OP_MIN = 3, OP_AVG = 4 };
/* device-side op kinds (the ncclDevRedOp_t subset used by the path) */
enum { DEV_SUM = 0, DEV_PROD = 1, DEV_MINMAX = 2, DEV_PREMULSUM = 3, DEV_SUMPOSTDIV = 4 };

int oracle_type_size(int dt) {
  switch (dt) {
    case DT_I8: case DT_U8: case DT_E4M3: case DT_E5M2: return 1;
    case DT_F16: case DT_BF16: return 2;
    case DT_I32: case DT_U32: case DT_F32: return 4;
    case DT_I64: case DT_U64: case DT_F64: return 8;
    default: return -1;
  }
}

/* ---------------- IEEE conversions (round-to-nearest-even) ---------------- */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float oracle_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff;
  if (exp == 0x1f) return u2f(sign | 0x7f800000u | (man << 13));
  if (exp == 0) {
    if (man == 0) return u2f(sign);
    /* subnormal: value = man * 2^-24 (exact in fp32) */
    float v = (float)man * 5.9604644775390625e-08f;
    return sign ? -v : v;
  }
  return u2f(sign | ((exp + 112) << 23) | (man << 13));
}

uint16_t oracle_f32_to_f16(float f) {
  uint32_t u = f2u(f);
  uint16_t sign = (uint16_t)((u >> 16) & 0x8000);
  uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return sign | 0x7e00 | (uint16_t)((a >> 13) & 0x3ff); /* NaN, quiet */
  if (a >= 0x477ff000u) return sign | 0x7c00; /* >= 65520 rounds to inf (also inf) */
  if (a < 0x38800000u) {                       /* below 2^-14: subnormal half (or zero) */
    /* value in units of 2^-24, rounded to nearest even */
    float v = u2f(a) * 16777216.0f;            /* exact scaling by 2^24 */
    float r = nearbyintf(v);                   /* default rounding mode = RNE */
    return sign | (uint16_t)r;
  }
  uint32_t exp = (a >> 23) - 112, man = a & 0x7fffff;
  uint32_t h = (exp << 10) | (man >> 13);
  uint32_t rem = man & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
  return sign | (uint16_t)h;
}

float oracle_bf16_to_f32(uint16_t b) { return u2f((uint32_t)b << 16); }

uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40); /* quiet NaN */
  u += 0x7fffu + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

/* OCP fp8: e4m3fn (bias 7, no inf, NaN = S.1111.111, max 448) and e5m2 (bias 15, IEEE-like). */
float oracle_fp8_to_f32(uint8_t v, int e5m2) {
  uint32_t sign = (v & 0x80) ? 1u : 0u;
  int ebits = e5m2 ? 5 : 4, mbits = e5m2 ? 2 : 3, bias = e5m2 ? 15 : 7;
  uint32_t exp = (v >> mbits) & ((1u << ebits) - 1), man = v & ((1u << mbits) - 1);
  float r;
  if (e5m2 && exp == 31) r = man ? NAN : INFINITY;
  else if (!e5m2 && exp == 15 && man == 7) r = NAN;
  else if (exp == 0) r = ldexpf((float)man, 1 - bias - mbits);
  else r = ldexpf((float)(man | (1u << mbits)), (int)exp - bias - mbits);
  return sign ? -r : r;
}

/* float -> fp8, RNE, saturating to the largest finite value (the __NV_SATFINITE mode that the
 * reference's fp8 functors use when converting the half result back, reduce_kernel.h:461-487). */
uint8_t oracle_f32_to_fp8(float f, int e5m2) {
  uint8_t sign = (f2u(f) >> 24) & 0x80;
  if (isnan(f)) return sign | 0x7f;
  int mbits = e5m2 ? 2 : 3, bias = e5m2 ? 15 : 7;
  float maxv = e5m2 ? 57344.0f : 448.0f;
  uint8_t maxcode = e5m2 ? 0x7b : 0x7e;
  float a = fabsf(f);
  if (a >= maxv) return sign | maxcode; /* saturate (includes inf) */
  /* quantum at this magnitude */
  int e;
  frexpf(a, &e); /* a = m * 2^e, m in [0.5,1) => unbiased exponent e-1 */
  int ue = e - 1;
  if (ue < 1 - bias) ue = 1 - bias; /* subnormal range */
  float q = ldexpf(1.0f, ue - mbits);
  float r = nearbyintf(a / q) * q; /* exact division by power of two; RNE */
  if (r >= maxv) return sign | maxcode;
  if (r == 0.0f) return sign;
  frexpf(r, &e);
  ue = e - 1;
  uint32_t code;
  if (ue < 1 - bias) { /* subnormal */
    code = (uint32_t)(r / ldexpf(1.0f, 1 - bias - mbits));
  } else {
    uint32_t man = (uint32_t)(r / ldexpf(1.0f, ue - mbits)) - (1u << mbits);
    code = ((uint32_t)(ue + bias) << mbits) | man;
  }
  return sign | (uint8_t)code;
}

/* ---------------- element access ---------------- */

static inline uint64_t ld(int dt, const void* p, size_t i) {
  switch (oracle_type_size(dt)) {
    case 1: return ((const uint8_t*)p)[i];
    case 2: return ((const uint16_t*)p)[i];
    case 4: return ((const uint32_t*)p)[i];
    default: return ((const uint64_t*)p)[i];
  }
}
static inline void st(int dt, void* p, size_t i, uint64_t v) {
  switch (oracle_type_size(dt)) {
    case 1: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case 2: ((uint16_t*)p)[i] = (uint16_t)v; break;
    case 4: ((uint32_t*)p)[i] = (uint32_t)v; break;
    default: ((uint64_t*)p)[i] = v; break;
  }
}
static inline int is_int(int dt) { return dt <= DT_U64; }
static inline uint64_t mask_of(int dt) {
  int b = 8 * oracle_type_size(dt);
  return b == 64 ? ~0ull : ((1ull << b) - 1);
}

/* small-float (f16/bf16/fp8) <-> f32 */
static inline float sf_to_f(int dt, uint64_t v) {
  switch (dt) {
    case DT_F16: return oracle_f16_to_f32((uint16_t)v);
    case DT_BF16: return oracle_bf16_to_f32((uint16_t)v);
    case DT_E4M3: return oracle_fp8_to_f32((uint8_t)v, 0);
    default: return oracle_fp8_to_f32((uint8_t)v, 1);
  }
}
/* Round an fp32 result of one half-precision operation back to T.
 * f16/bf16: one RNE rounding (equal to native __hadd/__hmul).
 * fp8: the reference computes in half (__hadd/__hmul on __half) then converts to fp8 with
 * saturation, so round to f16 first, then to fp8 (double rounding restated as-is). */
static inline uint64_t f_to_sf(int dt, float f) {
  switch (dt) {
    case DT_F16: return oracle_f32_to_f16(f);
    case DT_BF16: return oracle_f32_to_bf16(f);
    case DT_E4M3: return oracle_f32_to_fp8(oracle_f16_to_f32(oracle_f32_to_f16(f)), 0);
    default: return oracle_f32_to_fp8(oracle_f16_to_f32(oracle_f32_to_f16(f)), 1);
  }
}

/* ---------------- op mapping: hostToDevRedOp (src/enqueue.cc:2479-2583) ---------------- */

int oracle_host_to_dev_op(int op, int dt, int nranks, int* devop, uint64_t* arg) {
  int nbits = 8 * oracle_type_size(dt);
  if (nbits <= 0) return 4;
  uint64_t allBits = nbits == 64 ? ~0ull : ((1ull << nbits) - 1);
  uint64_t signBit = allBits ^ (allBits >> 1);
  *arg = 0;
  switch (op) {
    case OP_SUM: *devop = DEV_SUM; return 0;
    case OP_PROD: *devop = DEV_PROD; return 0;
    case OP_MIN:
    case OP_MAX:
      *devop = DEV_MINMAX;
      if (dt == DT_I8 || dt == DT_I32 || dt == DT_I64) *arg ^= signBit;
      if (op == OP_MAX) *arg ^= allBits;
      return 0;
    case OP_AVG:
      switch (dt) {
        case DT_I8: case DT_I32: case DT_I64:
          *devop = DEV_SUMPOSTDIV; *arg = ((uint64_t)nranks << 1) | 1; return 0;
        case DT_U8: case DT_U32: case DT_U64:
          *devop = DEV_SUMPOSTDIV; *arg = ((uint64_t)nranks << 1); return 0;
        case DT_F16: *devop = DEV_PREMULSUM; *arg = oracle_f32_to_f16((float)(1.0 / nranks)); return 0;
        case DT_BF16: *devop = DEV_PREMULSUM; *arg = oracle_f32_to_bf16((float)(1.0 / nranks)); return 0;
        case DT_E4M3: *devop = DEV_PREMULSUM; *arg = oracle_f32_to_fp8((float)(1.0 / nranks), 0); return 0;
        case DT_E5M2: *devop = DEV_PREMULSUM; *arg = oracle_f32_to_fp8((float)(1.0 / nranks), 1); return 0;
        case DT_F32: { float s = (float)(1.0 / nranks); *devop = DEV_PREMULSUM; *arg = f2u(s); return 0; }
        case DT_F64: { double s = 1.0 / nranks; *devop = DEV_PREMULSUM; memcpy(arg, &s, 8); return 0; }
      }
      return 4;
    default: return 4;
  }
}

/* ---------------- functors ---------------- */

/* fminf/fmaxf semantics (NaN-ignoring, reduce_kernel.h:409-410) with the signed-zero tie made
 * explicit: -0 is the smaller of (-0, +0). C leaves fmin(+0,-0) implementation-defined. */
static double omin(double x, double y) {
  if (isnan(x)) return y;
  if (isnan(y)) return x;
  if (x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}
static double omax(double x, double y) {
  if (isnan(x)) return y;
  if (isnan(y)) return x;
  if (x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}

static inline uint64_t pre_op(int dt, int devop, uint64_t arg, uint64_t x) {
  if (devop != DEV_PREMULSUM) return x;
  if (is_int(dt)) return (x * arg) & mask_of(dt);
  if (dt == DT_F32) return f2u(u2f((uint32_t)x) * u2f((uint32_t)arg));
  if (dt == DT_F64) { double a, s; memcpy(&a, &x, 8); memcpy(&s, &arg, 8); a *= s; uint64_t r; memcpy(&r, &a, 8); return r; }
  return f_to_sf(dt, sf_to_f(dt, x) * sf_to_f(dt, arg));
}

/* returns f(a, b) with a = pre-op'd local input, b = incoming accumulator */
static inline uint64_t reduce2(int dt, int devop, uint64_t arg, uint64_t a, uint64_t b) {
  int kind = (devop == DEV_PREMULSUM || devop == DEV_SUMPOSTDIV) ? DEV_SUM : devop;
  if (is_int(dt)) {
    uint64_t m = mask_of(dt);
    switch (kind) {
      case DEV_SUM: return (a + b) & m;
      case DEV_PROD: return (a * b) & m;
      default: return ((a ^ arg) & m) < ((b ^ arg) & m) ? a : b;
    }
  }
  int isMin = (arg & 1) == 0;
  if (dt == DT_F32) {
    float x = u2f((uint32_t)a), y = u2f((uint32_t)b), r;
    switch (kind) {
      case DEV_SUM: r = x + y; break;
      case DEV_PROD: r = x * y; break;
      default: r = (float)(isMin ? omin(x, y) : omax(x, y)); break;
    }
    return f2u(r);
  }
  if (dt == DT_F64) {
    double x, y, r; memcpy(&x, &a, 8); memcpy(&y, &b, 8);
    switch (kind) {
      case DEV_SUM: r = x + y; break;
      case DEV_PROD: r = x * y; break;
      default: r = isMin ? omin(x, y) : omax(x, y); break;
    }
    uint64_t u; memcpy(&u, &r, 8); return u;
  }
  float x = sf_to_f(dt, a), y = sf_to_f(dt, b), r;
  switch (kind) {
    case DEV_SUM: r = x + y; break;
    case DEV_PROD: r = x * y; break;
    default: r = (float)(isMin ? omin(x, y) : omax(x, y)); break;
  }
  return f_to_sf(dt, r);
}

/* SumPostDiv: integer divide of the wrapped sum by nranks (reduce_kernel.h:936-966): magnitude
 * quotient, sign restored — i.e. truncation toward zero for signed types. */
static inline uint64_t post_op(int dt, int devop, uint64_t arg, uint64_t x) {
  if (devop != DEV_SUMPOSTDIV || !is_int(dt)) return x;
  uint64_t m = mask_of(dt);
  int isSigned = (int)(arg & 1);
  uint64_t divisor = arg >> 1;
  uint64_t sign = m ^ (m >> 1);
  int neg = isSigned && (x & sign);
  uint64_t xabs = neg ? ((0 - x) & m) : x;
  uint64_t q = xabs / divisor;
  return neg ? ((0 - q) & m) : q;
}

/* Fold element i across ranks in ring order starting at `first`:
 *   acc = pre(x[first]); for k = 1..n-1: acc = f(pre(x[(first+k)%n]), acc); return post(acc). */
static inline uint64_t fold_elem(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t idx,
                                 int first) {
  uint64_t acc = pre_op(dt, devop, arg, ld(dt, in[first], idx));
  for (int k = 1; k < n; k++) {
    int r = (first + k) % n;
    acc = reduce2(dt, devop, arg, pre_op(dt, devop, arg, ld(dt, in[r], idx)), acc);
  }
  return post_op(dt, devop, arg, acc);
}

/* ---------------- collectives ---------------- */

/* AllReduce: out[i] for i in [0,count). Rank chunk rc = alignUp(divUp(count,n), 16/sizeof(T))
 * (all_reduce.h:38 with one channel and one loop); chunk c is owned by rank c and folded from c+1.
 * Returns 0 on success, 4 on invalid argument. */
int oracle_all_reduce(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t count, void* out) {
  int ts = oracle_type_size(dt);
  if (ts <= 0 || n <= 0) return 4;
  if (n == 1) { /* nranks==1 path (src/device/onerank.cu:49-110): copy, or PreMulSum kernel */
    for (size_t i = 0; i < count; i++) st(dt, out, i, post_op(dt, devop, arg, pre_op(dt, devop, arg, ld(dt, in[0], i))));
    return 0;
  }
  size_t epp = (size_t)(16 / ts);
  size_t rc = (count + n - 1) / n;
  rc = (rc + epp - 1) / epp * epp;
  /* elements are independent: OpenMP over them keeps full-config sizes (C2..C5) checkable in seconds */
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    int owner = (int)(i / rc);
    st(dt, out, i, fold_elem(dt, devop, arg, n, in, i, (owner + 1) % n));
  }
  return 0;
}

/* ---- the reference's RING AllReduce partition at full size (more than one channel and loop) ----
 * NCCL cuts a large AllReduce into channel parts and each part into loops of n chunks; a chunk's elements are
 * finalised by the ring position of the chunk INSIDE ITS LOOP, so which rank's input an element's fold starts
 * from depends on this partition. The three protocols run the same ring (runRing<T, RedOp, Proto>,
 * src/device/all_reduce.h:13-83, 229-233, 763-781) on different partitions. Restated for ONE task on a
 * communicator of `nchannels` channels, protocol `proto` (0 LL, 1 LL128, 2 SIMPLE: NCCL_PROTO_* ids) with that
 * protocol's buffer of `buffsize` bytes (0 = its default: NCCL_LL_BUFFSIZE 8 lines x 512 threads x 8 steps x
 * 16 B = 512 KiB, NCCL_LL128_BUFFSIZE 120 x 640 x 8 x 8 B, NCCL_BUFFSIZE 4 MiB; src/init.cc:810-827):
 *   channel count   topoGetAlgoInfo, RING: nc = nchannels, decremented while nBytes < nc * nt * threshold
 *                   (src/enqueue.cc:2070-2097) with nt / threshold = 512 / 64 (SIMPLE, NVLink-class bandwidth,
 *                   tuning.cc:244-247, 591), 512 / 8 x nranks (LL, tuning.cc:253-254, 589, 593), 640 / 8
 *                   (LL128, tuning.cc:255-257, 590)
 *   parts (CBD)     scheduleCollTasksToPlan for a lone task (channelId 0, no traffic yet): AllReduce moves 2 bytes
 *                   of traffic per byte, 8 under LL (enqueue.cc:461, 658); cells of 32 KiB of traffic (16 KiB of
 *                   data, 4 KiB under LL), lo / mid / hi channel parts: src/enqueue.cc:576-757, trafficPerByte
 *                   :91-94; the part of channel c: device.h:337-361
 *   chunk           calcCollChunking, RING: stepSize = buffsize / NCCL_STEPS (8); SIMPLE x ALLREDUCE_CHUNKSTEPS
 *                   (4) in 512-byte grains, LL / 2 in 16-byte grains, LL128 x 15/16 (data elements per 128-byte
 *                   line) in 1920-byte grains: src/enqueue.cc:2222-2227, 2321; collectives.h:19-20;
 *                   device.h:328-334, 97-117
 *   loops           runRing: loopCount = n * chunkCount; the last loop re-cuts chunkCount to
 *                   alignUp(divUp(rem, n), 16 / sizeof(T)): src/device/all_reduce.h:21-38
 * plan[0..4] = {channels, countLo, countMid, countHi, chunk elements}. */
static size_t div_up(size_t a, size_t b) { return (a + b - 1) / b; }

int oracle_ring_nccl_plan_proto(size_t count, int ts, int nranks, int nchannels, int proto, size_t buffsize,
                                uint64_t* plan) {
  if (ts <= 0 || nranks <= 0 || nchannels <= 0 || count == 0 || proto < 0 || proto > 2) return 4;
  static const size_t defBuff[3] = {(size_t)8 * 512 * 8 * 16, (size_t)120 * 640 * 8 * 8, (size_t)1 << 22};
  static const size_t grain[3] = {16, 1920, 512};
  if (buffsize == 0) buffsize = defBuff[proto];
  /* channel count (enqueue.cc:2093-2096) */
  const size_t nBytes = count * (size_t)ts;
  const size_t nt = proto == 1 ? 640 : 512;
  const size_t thr = proto == 0 ? (size_t)8 * nranks : proto == 1 ? 8 : 64;
  int nc = nchannels;
  while (nBytes < (size_t)nc * nt * thr) {
    if (nc >= 2) nc--;
    else break;
  }
  /* CBD (enqueue.cc:580-604, 617-620, 657-701) */
  const size_t minTraffic = (size_t)32 << 10;
  const size_t trafficPerByte = proto == 0 ? 8 : 2;
  size_t trafficBytes = count * (size_t)ts * trafficPerByte;
  if (trafficBytes < minTraffic) trafficBytes = minTraffic;
  const size_t trafficPerChannel = div_up(trafficBytes / (size_t)nc, 16) * 16;
  const size_t cellSize = div_up(div_up(minTraffic, trafficPerByte), 16) * 16;
  const size_t elementsPerCell = cellSize / (size_t)ts;
  const size_t cells = div_up(count * (size_t)ts, cellSize);
  const size_t trafficPerCell = cellSize * trafficPerByte;
  size_t cellsPerChannel = div_up(trafficPerChannel, trafficPerCell);
  if (cellsPerChannel > cells) cellsPerChannel = cells;
  /* the traffic per channel divides by the task's channel count nc, the bounds below compare with the
   * communicator's (nMaxChannels[kind] = comm->nChannels, enqueue.cc:583) */
  size_t cellsLo;
  if (nchannels == 1) cellsLo = cells; /* channelId + 1 == nMaxChannels */
  else {
    cellsLo = div_up(trafficPerChannel, trafficPerCell);
    if (cellsLo > cells) cellsLo = cells;
  }
  long nMid = (long)((cells - cellsLo) / cellsPerChannel);
  size_t cellsHi = (cells - cellsLo) % cellsPerChannel;
  long used = (cellsLo != 0) + nMid + (cellsHi != 0);
  if (nchannels < used) { /* overflowed the channels */
    nMid = nchannels - 2;
    cellsPerChannel = (cells - cellsLo) / (size_t)(nMid + 1);
    cellsHi = cellsPerChannel + (cells - cellsLo) % (size_t)(nMid + 1);
  }
  if (cellsHi == 0 && nMid != 0) {
    cellsHi = cellsPerChannel;
    nMid -= 1;
  }
  /* cellsLo == 0 cannot happen for the first task of a plan (count > 0) */
  size_t countMid = nMid != 0 ? cellsPerChannel * elementsPerCell : 0;
  size_t countLo = cellsLo * elementsPerCell;
  size_t countHi = cellsHi * elementsPerCell;
  const size_t excess = cells * elementsPerCell - count;
  if (countHi != 0) countHi -= excess;
  else countLo -= excess;
  used = (countLo != 0) + nMid + (cellsHi != 0);
  /* chunk (enqueue.cc:2222-2227, 2321), in grains; the device's chunkCount = grains x grain / sizeof(T) */
  const size_t step = buffsize / 8;
  size_t chunkBytes = proto == 2 ? step * 4 : proto == 0 ? step / 2 : step / 16 * 15;
  const size_t grains = chunkBytes / grain[proto];
  if (grains == 0) return 4; /* a zero chunk never advances (the reference loops forever) */
  plan[0] = (uint64_t)used;
  plan[1] = countLo;
  plan[2] = countMid;
  plan[3] = countHi;
  plan[4] = grains * (grain[proto] / (size_t)ts);
  return 0;
}

int oracle_ring_nccl_plan(size_t count, int ts, int nranks, int nchannels, size_t buffsize, uint64_t* plan) {
  return oracle_ring_nccl_plan_proto(count, ts, nranks, nchannels, 2, buffsize, plan);
}

/* AllReduce in the reference's RING order at full size: element e of channel part [off, off + cnt) in loop
 * l = (e - off) / (n * chunk) lies in chunk q of that loop and is finalised by ring position q, i.e. folded from
 * q + 1 (all_reduce.h:42-81; ring index = rank). */
int oracle_all_reduce_ring_nccl_proto(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t count,
                                      void* out, int nchannels, int proto, size_t buffsize) {
  int ts = oracle_type_size(dt);
  if (ts <= 0 || n <= 0) return 4;
  if (count == 0) return 0;
  if (n == 1) return oracle_all_reduce(dt, devop, arg, n, in, count, out);
  uint64_t plan[5];
  if (oracle_ring_nccl_plan_proto(count, ts, n, nchannels, proto, buffsize, plan)) return 4;
  const int nch = (int)plan[0];
  const size_t epp = (size_t)(16 / ts);
  for (int c = 0; c < nch; c++) {
    size_t off, cnt; /* ncclCollCbdPart (device.h:337-361) with channelLo = 0, channelHi = nch - 1 */
    if (c == 0) { off = 0; cnt = plan[1]; }
    else if (c == nch - 1) { off = plan[1] + (size_t)(nch - 2) * plan[2]; cnt = plan[3]; }
    else { off = plan[1] + (size_t)(c - 1) * plan[2]; cnt = plan[2]; }
    size_t chunk = plan[4];
    const size_t loopCount = (size_t)n * chunk;
    for (size_t eo = 0; eo < cnt; eo += loopCount) {
      const size_t rem = cnt - eo;
      if (rem < loopCount) chunk = div_up(div_up(rem, (size_t)n), epp) * epp;
      const size_t len = rem < loopCount ? rem : loopCount;
#pragma omp parallel for schedule(static)
      for (size_t j = 0; j < len; j++) {
        const int q = (int)(j / chunk);
        const size_t i = off + eo + j;
        st(dt, out, i, fold_elem(dt, devop, arg, n, in, i, (q + 1) % n));
      }
    }
  }
  return 0;
}

int oracle_all_reduce_ring_nccl(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t count,
                                void* out, int nchannels, size_t buffsize) {
  return oracle_all_reduce_ring_nccl_proto(dt, devop, arg, n, in, count, out, nchannels, 2, buffsize);
}

/* AllReduce over the reference's intra-node TREE (NCCL_ALGO=TREE): a chain with root 0 and leaf n-1
 * (src/graph/connect.cc:53-63, treeIntra = 0..n-1): the leaf sends pre(x[n-1]), rank k folds
 * red(pre(x[k]), acc) on the way up (all_reduce.h:86-118 runTreeUpDown), the root applies post and the
 * result is broadcast back down. Every element folds in the order n-1, n-2, ..., 0. */
int oracle_all_reduce_chain(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t count, void* out) {
  if (oracle_type_size(dt) <= 0 || n <= 0) return 4;
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    uint64_t acc = pre_op(dt, devop, arg, ld(dt, in[n - 1], i));
    for (int r = n - 2; r >= 0; r--) acc = reduce2(dt, devop, arg, pre_op(dt, devop, arg, ld(dt, in[r], i)), acc);
    st(dt, out, i, post_op(dt, devop, arg, acc));
  }
  return 0;
}

/* ReduceScatter: out[d][j] = fold over ranks of in[r][d*recvcount + j], from d+1 (reduce_scatter.h:34-55). */
int oracle_reduce_scatter(int dt, int devop, uint64_t arg, int n, const void* const* in, size_t recvcount,
                          void* const* out) {
  if (oracle_type_size(dt) <= 0 || n <= 0) return 4;
  for (int d = 0; d < n; d++) {
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < recvcount; j++)
      st(dt, out[d], j, fold_elem(dt, devop, arg, n, in, (size_t)d * recvcount + j, (d + 1) % n));
  }
  return 0;
}

/* Reduce to root: chain root+1 -> ... -> root (reduce.h:34-52). */
int oracle_reduce(int dt, int devop, uint64_t arg, int n, int root, const void* const* in, size_t count, void* out) {
  if (oracle_type_size(dt) <= 0 || n <= 0 || root < 0 || root >= n) return 4;
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) st(dt, out, i, fold_elem(dt, devop, arg, n, in, i, (root + 1) % n));
  return 0;
}

/* ---------------- synthetic inputs: splitmix64 counter PRNG ---------------- */

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

/* kind 0: uniform in [-1,1) (24-bit grid, rounded RNE to T for small floats; full range for ints,
 *         with INT_MIN/INT_MAX-style extremes at i%1024==1 / ==2);
 * kind 1: dyadic k/256 with |k| <= 1024 (exact sums for fp32 up to 2^14 terms). */
/* elements [start, start + count) of the sequence oracle_fill produces (out[0] = element start) */
void oracle_fill_at(int dt, uint64_t seed, size_t start, size_t count, void* out, int kind) {
#pragma omp parallel for schedule(static)
  for (size_t j = 0; j < count; j++) {
    const size_t i = start + j;
    uint64_t r = splitmix64(seed * 0x100000001b3ull ^ (uint64_t)i);
    if (is_int(dt)) {
      uint64_t m = mask_of(dt), sign = m ^ (m >> 1);
      uint64_t v = r & m;
      if (i % 1024 == 1) v = sign;       /* INT_MIN bit pattern for signed types */
      else if (i % 1024 == 2) v = sign - 1; /* INT_MAX */
      st(dt, out, j, v);
      continue;
    }
    double x;
    if (kind == 1) x = (double)((int64_t)(r % 2049) - 1024) / 256.0;
    else x = (double)((int64_t)(r >> 40) - (1ll << 23)) / (double)(1 << 23);
    switch (dt) {
      case DT_F32: st(dt, out, j, f2u((float)x)); break;
      case DT_F64: { uint64_t u; memcpy(&u, &x, 8); st(dt, out, j, u); break; }
      default: st(dt, out, j, f_to_sf(dt, (float)x)); break;
    }
  }
}

void oracle_fill(int dt, uint64_t seed, size_t count, void* out, int kind) { oracle_fill_at(dt, seed, 0, count, out, kind); }

/* ---------------- naive OpenMP CPU baseline ---------------- */

/* fp32 sum AllReduce of n host buffers into `out`, same fold order as oracle_all_reduce. Returns the
 * number of threads used. */
int oracle_cpu_allreduce_f32(int n, const float* const* in, size_t count, float* out, int nthreads) {
  size_t rc = (count + n - 1) / n;
  rc = (rc + 3) / 4 * 4;
  int used = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#pragma omp single
    used = omp_get_num_threads();
  }
#endif
  for (int c = 0; c < n; c++) {
    size_t lo = (size_t)c * rc, hi = lo + rc < count ? lo + rc : count;
    if (lo >= count) break;
    int first = (c + 1) % n;
#pragma omp parallel for simd schedule(static)
    for (size_t i = lo; i < hi; i++) {
      float acc = in[first][i];
      for (int k = 1; k < n; k++) acc = in[(first + k) % n][i] + acc;
      out[i] = acc;
    }
  }
  return used;
}
