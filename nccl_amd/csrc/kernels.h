// kernels.h — gfx950 device code of the reduction engine (templates; instantiated per element type in
// kern_<type>.hip so the kernels build in parallel) + the typed launch templates.
//
// Replaces the reference's device tree src/device/ (runRing in all_reduce.h / reduce_scatter.h /
// all_gather.h / reduce.h, Primitives<ProtoSimple> in prims_simple.h, reduceCopy in
// common_kernel.h, oneRankReduce in onerank.cu). It is NOT a ring: every MI355X of the node has a
// direct xGMI link to every other one, so the buffer is cut into nRanks blocks (block q owned by
// rank q) and each rank
//   A  scatters block q of its input to owner q's staging (n-1 remote write streams, one per link),
//   B  folds the n contributions of its own block in the reference's ring order (owner+1, ...,
//      owner; per-hop rounding to T) and pushes the result to every peer's all-gather staging,
//   C  copies the n-1 gathered blocks from its own staging into the output.
// Each workgroup is an independent "channel" (reference: one CTA per channel) that pipelines its
// part of every block in slices through nSlots staging slots per peer, with per-connection credit
// counters exactly like the reference's head/tail protocol (prims_simple.h:100-173), but
// bidirectional over all 7 links at once instead of one ring neighbour.
//
// Besides this staged kernel (collKernel, with its one-shot variant COLL_AR1) the file holds
//   llKernel   the LL protocol for small AllReduces and group batches (flag-in-data lines, no fences),
//   symKernel  the zero-copy kernels for buffers in symmetric windows (peers' buffers pulled directly),
//   oneRankKernel (PreMulSum at nRanks == 1; the nRanks == 1 copy lives in kernels.hip).
//
// Memory model: remote payload = `global_store_dwordx4 ... sc0 sc1` (system-scope
// write-through) into the peer's UNCACHED staging; every storing wave drains (s_waitcnt vmcnt(0)),
// the workgroup barriers, one lane issues a system release fence and then a system-scope flag
// store. The consumer polls its local flag with system-scope loads (one wave, s_sleep between polls,
// bounded by NCCL_AMD_SPIN_TIMEOUT_MS and the host abort word), then one system acquire
// (buffer_inv sc0 sc1), vmcnt(0), barrier, plain loads.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "core.h"
#include "numerics.h"

namespace ncclamd {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 512;  // 8 waves of 64 per channel workgroup
// Several ranks on one GPU (NCCL_MULTI_RANK_GPU_ENABLE) need every channel of every rank resident at
// once: the host caps channels at 2 workgroups per CU (chanCap), so each channel kernel must fit two
// 512-thread workgroups per CU = 4 waves per SIMD, i.e. at most 128 VGPRs. The attribute makes the
// compiler hold that budget (tests/test_occupancy.py checks the build's resource report).
#define kCoResident __attribute__((amdgpu_waves_per_eu(4)))

// NCCL_AMD_KERNEL_LOG=<path>: each distinct kernel this process launches is named once in that file
// ("<kernel> grid=<workgroups> block=<threads>", kernels.hip kernelLogNote) — how bench.py names the kernel
// its roofline measures, from the run itself. Off: one predictable branch per launch.
extern bool gKernelLog;
void kernelLogNote(const void* fn, unsigned grid, unsigned block);
#define NCCL_AMD_LAUNCH(K, G, B, SH, ST, ...)                                                  \
  do {                                                                                          \
    if (::ncclamd::gKernelLog) ::ncclamd::kernelLogNote((const void*)(K), (G).x, (B).x);      \
    hipLaunchKernelGGL(K, G, B, SH, ST, __VA_ARGS__);                                           \
  } while (0)

// ------------------------------------------------------------------------------------ primitives

__device__ __forceinline__ uint64_t clockTicks() { return __builtin_amdgcn_s_memrealtime(); }

// The stores are inline asm (the compiler has no builtin for a write-through system-scope store), so the
// compiler's hazard recognizer cannot see them: each one carries its own trailing wait states, or a VALU /
// LDS write that reuses its address or data VGPRs right behind it can be picked up by the store (seen as
// pointer-valued garbage in 16-byte-pack-sized holes of the uint32/uint64 kernels once register allocation
// placed such a write there).
__device__ __forceinline__ void storeRemote(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void drainStores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Bulk remote stores (staging slots, AG pushes) as compiler-visible buffer stores with the same cache policy
// (sc0 sc1: system-scope write-through). The compiler cannot see an inline-asm store, and on gfx9 stores
// count in vmcnt like loads: a copy loop of asm stores therefore ends every batch with vmcnt(0), i.e. waits
// for its own stores' completion before the next loads go out. With intrinsic stores the waits cover only
// the loads. The destination base is wave-uniform (readfirstlane makes that explicit); offsets are 32-bit
// (a slot or slice is far below 4 GiB).
#ifndef NCCL_AMD_BUFFER_STORES
#define NCCL_AMD_BUFFER_STORES 1
#endif
constexpr int kSysWriteThrough = 1 | 16;  // buffer cache policy bits: sc0 (bit 0) | sc1 (bit 4)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t remoteRsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, -1, 0x00020000);
}
__device__ __forceinline__ void storeRemoteAt(__amdgpu_buffer_rsrc_t r, uint32_t byteOff, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byteOff, 0, kSysWriteThrough);
}

// This rank's own outputs (phase B's fold result, phase C's gathered blocks, the symmetric kernels' results):
// NCCL_AMD_LOCAL_WT=1 writes them with the same system-scope write-through buffer stores as the remote ones
// instead of global nontemporal stores (A/B knob; the nRanks==1 copy measured the difference).
// `base` is the batch's wave-uniform first pack, so offsets stay small at any buffer size.
#ifndef NCCL_AMD_LOCAL_WT
#define NCCL_AMD_LOCAL_WT 0
#endif
struct LocalStore {
  __amdgpu_buffer_rsrc_t r;
  u32x4* d;
  __device__ __forceinline__ LocalStore(void* dst, uint64_t base) : d((u32x4*)dst + base) {
    if (NCCL_AMD_LOCAL_WT) r = remoteRsrc(d);
  }
  __device__ __forceinline__ void put(uint32_t k, u32x4 v) {  // pack base + k
    if (NCCL_AMD_LOCAL_WT) __builtin_amdgcn_raw_buffer_store_b128(v, r, k * 16u, 0, kSysWriteThrough);
    else __builtin_nontemporal_store(v, d + k);
  }
};

// One element stored system-scope write-through (tails and unaligned ranges of published data).
template <typename T>
__device__ __forceinline__ void storeRemoteElt(T* p, T v) {
  if constexpr (sizeof(T) == 1) {
    uint32_t x = 0;
    __builtin_memcpy(&x, &v, 1);
    asm volatile("global_store_byte %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
  } else if constexpr (sizeof(T) == 2) {
    uint32_t x = 0;
    __builtin_memcpy(&x, &v, 2);
    asm volatile("global_store_short %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
  } else if constexpr (sizeof(T) == 4) {
    uint32_t x;
    __builtin_memcpy(&x, &v, 4);
    asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
  } else {
    uint64_t x;
    __builtin_memcpy(&x, &v, 8);
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
  }
}

__device__ __forceinline__ uint64_t loadFlag(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void storeFlag(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void reportError(const DevComm& dc, uint32_t code) {
  uint32_t expected = 0;
  __hip_atomic_compare_exchange_strong(dc.errorWord, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block-wide state kept in LDS.
struct ChanState {
  uint64_t ctr[CTR_KINDS][NCCL_AMD_MAX_RANKS];
  int abort;
};


// Kernel-kind mismatch probe. Every rank must run the same kernel for one collective; the staged and
// the registered zero-copy kernels exchange different flags, so ranks that disagree (a registration that failed
// on one rank only, e.g. under graph capture) would each wait for a signal the other never sends until the spin
// timeout. A waiting lane whose peer has meanwhile posted a flag of the OTHER kernel kind on this channel beyond
// what this rank has consumed has proof of the disagreement: while this rank is blocked in op k on channel c,
// that peer cannot have finished op k on c (it needs this rank's signals of op k), so its newer flag of the other
// kind belongs to op k itself. The wait's own flag is read again after the probe (the peer's op-k signals complete
// before its next kernel starts), so a peer that merely moved on is never taken for a mismatch. Checked on the slow
// path only (every 256 polls): no cost while flags arrive.
//   staged kernels: peer's SYM_ENTER[c] > this channel's symmetric epoch (counters[c][CTR_SYM][0]);
//   symmetric kernels (ENTER wait): peer's RS_READY / AG_READY / PULL_READY[c] > what this rank consumed.
// PROBE_STAGED: flag[0] against `epoch` (one load per lane: staged kernels run at the 128-VGPR co-residency cap);
// PROBE_SYM: flag[k] against seen[k][peer], k < 3.
enum ProbeKind { PROBE_NONE = 0, PROBE_STAGED = 1, PROBE_SYM = 2 };
struct WaitProbe {
  const uint64_t* flag[3];  // the other kind's flag words of this channel, indexed by peer
  const uint64_t* seen[3];  // per-peer counts this rank consumed (PROBE_SYM)
  uint64_t epoch;           // this channel's symmetric epoch (PROBE_STAGED)
};
template <int PROBE>
__device__ __forceinline__ bool probeMismatch(const WaitProbe& pr, int lane) {
  if constexpr (PROBE == PROBE_STAGED) return loadFlag(pr.flag[0] + lane) > pr.epoch;
  bool ev = false;
#pragma unroll
  for (int k = 0; k < 3; k++) ev |= loadFlag(pr.flag[k] + lane) > pr.seen[k][lane];
  return ev;
}

// Wave 0 waits until every selected flag word reaches its target (target[r] == 0: no wait on r).
// ACQ: follow with a system-scope acquire (needed before reading data the flags publish; not for
// credit/ack words, which guard no data). All threads must call it (it ends in a barrier).
// PROBE / probe: the kernel-kind mismatch probe above.
template <int PROBE = PROBE_NONE>
__device__ bool waitAll(const DevComm& dc, ChanState& st, const uint64_t* flagBase, const uint64_t* target,
                        bool ACQ, const WaitProbe* probe = nullptr) {
  if (threadIdx.x < 64) {
    int lane = threadIdx.x;
    bool need = lane < dc.nRanks && target[lane] != 0;
    uint64_t t0 = 0;
    uint32_t iter = 0;
    while (true) {
      bool ok = !need || loadFlag(flagBase + lane) >= target[lane];
      if (__all(ok)) break;
      if (iter == 0) t0 = clockTicks();
      __builtin_amdgcn_s_sleep(1);
      if ((++iter & 255) == 0) {
        bool bad = false;
        bool mismatch = false;
        if (PROBE != PROBE_NONE && need && probeMismatch<PROBE>(*probe, lane)) {
          __atomic_thread_fence(__ATOMIC_ACQUIRE);
          mismatch = loadFlag(flagBase + lane) < target[lane];  // still missing after the other kind's flag
        }
        if (__hip_atomic_load(dc.abortFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          if (lane == 0) reportError(dc, DERR_ABORT);
          bad = true;
        } else if (__any(mismatch)) {
          if (mismatch) reportError(dc, DERR_MISMATCH);
          bad = true;
        } else if (__hip_atomic_load(dc.errorWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          bad = true;  // another workgroup already failed: stop waiting
        } else if (clockTicks() - t0 > dc.timeoutTicks) {
          if (lane == 0) reportError(dc, DERR_TIMEOUT);
          bad = true;
        }
        if (bad) {
          if (lane == 0) st.abort = 1;
          break;
        }
      }
    }
    if (ACQ && lane == 0) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // buffer_inv sc0 sc1 (system acquire)
    drainStores();
  }
  __syncthreads();
  return st.abort == 0;
}

// Every wave drains its memory operations, then wave-0 lane i stores val[i] into ptr[i] (val 0 = skip)
// with a system-scope store. REL: precede with a system release fence (publishing data); without it
// the stores are credits/acks: our loads of the consumed slot have completed (vmcnt(0)) and nothing
// we wrote needs to be visible.
__device__ void signalAll(uint64_t* const* ptr, const uint64_t* val, int nsig, bool REL) {
  drainStores();
  __syncthreads();
  if (threadIdx.x < 64) {
    int lane = threadIdx.x;
    if (REL) {
      __atomic_thread_fence(__ATOMIC_RELEASE);  // buffer_wbl2 sc0 sc1 + vmcnt(0)
      drainStores();                            // kept explicit: see MI355X_MICROARCH "Compiler hazard"
    }
    if (lane < nsig && val[lane] != 0) storeFlag(ptr[lane], val[lane]);
  }
}

// ------------------------------------------------------------------------------------ data movement

// 16-byte packs each thread keeps in flight in copyRange: 8 x 16 B x 512 threads = 64 KiB per channel, enough
// to keep one CU's share of HBM (and, on the 8-GPU node, its xGMI writes) busy at moderate channel counts.
#ifndef NCCL_AMD_COPY_UNROLL
#define NCCL_AMD_COPY_UNROLL 8
#endif
constexpr int kCopyUnroll = NCCL_AMD_COPY_UNROLL;
// 16-byte packs per batch of the fold (types wider than one byte); each has its successor's loads in flight.
#ifndef NCCL_AMD_FOLD_UNROLL
#define NCCL_AMD_FOLD_UNROLL 4
#endif
constexpr int kFoldUnroll = NCCL_AMD_FOLD_UNROLL;
#ifndef NCCL_AMD_FOLD_UNROLL_SWAR
#define NCCL_AMD_FOLD_UNROLL_SWAR 2
#endif
#ifndef NCCL_AMD_FOLD_UNROLL_1B
#define NCCL_AMD_FOLD_UNROLL_1B 2
#endif
constexpr int kFoldUnrollSwar = NCCL_AMD_FOLD_UNROLL_SWAR;
constexpr int kFoldUnroll1B = NCCL_AMD_FOLD_UNROLL_1B;
#ifndef NCCL_AMD_FOLD_REPACK
#define NCCL_AMD_FOLD_REPACK 1
#endif
// foldRange: the next batch's first source loaded while the current batch's last source folds (1), or after the
// batch's stores (0, round 5's order)
#ifndef NCCL_AMD_FOLD_PREFETCH
#define NCCL_AMD_FOLD_PREFETCH 1
#endif

// Copy [0,nbytes) from src to dst. Both 16-byte aligned when `aligned`; nbytes multiple of sizeof(T).
template <typename T, bool REMOTE>
__device__ __forceinline__ void copyRange(void* dst, const void* src, uint64_t nbytes, bool aligned) {
  if (aligned) {
    uint64_t npk = nbytes >> 4;
    const u32x4* s = (const u32x4*)src;
    u32x4* d = (u32x4*)dst;
    constexpr int U = kCopyUnroll;
    uint64_t i = threadIdx.x;
    for (; i + (U - 1) * kThreads < npk; i += U * kThreads) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * kThreads);
      LocalStore ls(dst, i - threadIdx.x);
      // the buffer resource is rebased on every batch (its wave-uniform first pack), so the 32-bit store
      // offsets stay below U * kThreads * 16 bytes whatever the range's size (a symmetric-window part can
      // exceed 4 GiB with a low channel cap)
      __amdgpu_buffer_rsrc_t rd;
      if (REMOTE && NCCL_AMD_BUFFER_STORES) rd = remoteRsrc(d + (i - threadIdx.x));
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (REMOTE && NCCL_AMD_BUFFER_STORES) storeRemoteAt(rd, (uint32_t)((threadIdx.x + u * kThreads) * 16), v[u]);
        else if (REMOTE) storeRemote(d + i + u * kThreads, v[u]);
        else ls.put(threadIdx.x + u * kThreads, v[u]);
      }
    }
    for (; i < npk; i += kThreads) {
      u32x4 v = __builtin_nontemporal_load(s + i);
      if (REMOTE && NCCL_AMD_BUFFER_STORES) storeRemoteAt(remoteRsrc(d + (i - threadIdx.x)), threadIdx.x * 16u, v);
      else if (REMOTE) storeRemote(d + i, v);
      else __builtin_nontemporal_store(v, d + i);
    }
    uint64_t done = npk << 4;
    uint64_t tail = (nbytes - done) / sizeof(T);
    if (threadIdx.x < tail) {
      const T* st = (const T*)((const char*)src + done);
      T* dt = (T*)((char*)dst + done);
      if (REMOTE) storeRemoteElt(dt + threadIdx.x, st[threadIdx.x]);
      else dt[threadIdx.x] = st[threadIdx.x];
    }
  } else {
    uint64_t n = nbytes / sizeof(T);
    const T* s = (const T*)src;
    T* d = (T*)dst;
    for (uint64_t i = threadIdx.x; i < n; i += kThreads) {
      if (REMOTE) storeRemoteElt(d + i, s[i]);
      else d[i] = s[i];
    }
  }
}

// One source copied to several destinations with ONE read of it: an optional local copy (dstLocal, plain stores)
// and nPush remote copies (system-scope write-through stores, one buffer resource per destination and batch).
// copyRange per destination read the source once per destination — nontemporal loads do not keep it in L2, so
// the AllGather publish read its block n times from HBM (PMC at n = 2: 2.96 S per rank instead of 2.5 S,
// profiles/pmc_traffic.json) and the one-shot publish n - 1 times.
template <typename T>
__device__ __forceinline__ void copyRangeMulti(char* dstLocal, char* const* dstPush, int nPush, const void* src,
                                               uint64_t nbytes, bool aligned) {
  if (nPush == 1 && !dstLocal) return copyRange<T, true>(dstPush[0], src, nbytes, aligned);  // one destination:
  if (nPush == 0) return dstLocal ? copyRange<T, false>(dstLocal, src, nbytes, aligned) : void();  // the plain copy
  if (aligned) {
    const uint64_t npk = nbytes >> 4;
    const u32x4* s = (const u32x4*)src;
    constexpr int U = kCopyUnroll;
    uint64_t i = threadIdx.x;
    for (; i + (U - 1) * kThreads < npk; i += U * kThreads) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * kThreads);
      if (dstLocal) {
        LocalStore ls(dstLocal, i - threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; u++) ls.put(threadIdx.x + u * kThreads, v[u]);
      }
      for (int p = 0; p < nPush; p++) {
        u32x4* d = (u32x4*)dstPush[p];
        if (NCCL_AMD_BUFFER_STORES) {
          const __amdgpu_buffer_rsrc_t rd = remoteRsrc(d + (i - threadIdx.x));
#pragma unroll
          for (int u = 0; u < U; u++) storeRemoteAt(rd, (uint32_t)((threadIdx.x + u * kThreads) * 16), v[u]);
        } else {
#pragma unroll
          for (int u = 0; u < U; u++) storeRemote(d + i + u * kThreads, v[u]);
        }
      }
    }
    for (; i < npk; i += kThreads) {
      const u32x4 v = __builtin_nontemporal_load(s + i);
      if (dstLocal) __builtin_nontemporal_store(v, (u32x4*)dstLocal + i);
      for (int p = 0; p < nPush; p++) {
        u32x4* d = (u32x4*)dstPush[p];
        if (NCCL_AMD_BUFFER_STORES) storeRemoteAt(remoteRsrc(d + (i - threadIdx.x)), threadIdx.x * 16u, v);
        else storeRemote(d + i, v);
      }
    }
    const uint64_t done = npk << 4;
    const uint64_t tail = (nbytes - done) / sizeof(T);
    if (threadIdx.x < tail) {
      const T x = ((const T*)((const char*)src + done))[threadIdx.x];
      if (dstLocal) ((T*)(dstLocal + done))[threadIdx.x] = x;
      for (int p = 0; p < nPush; p++) storeRemoteElt((T*)(dstPush[p] + done) + threadIdx.x, x);
    }
  } else {
    const uint64_t n = nbytes / sizeof(T);
    const T* s = (const T*)src;
    for (uint64_t i = threadIdx.x; i < n; i += kThreads) {
      const T x = s[i];
      if (dstLocal) ((T*)dstLocal)[i] = x;
      for (int p = 0; p < nPush; p++) storeRemoteElt((T*)dstPush[p] + i, x);
    }
  }
}

template <typename T>
union PackU {
  u32x4 v;
  T e[16 / sizeof(T)];
};

// fp8 fold of one 16-byte pack in f32 (numerics.h fp8Decode4 / fp8RoundF / fp8Encode4): the accumulator lives as
// the f32 values of its codes, each hop rounded to the value the per-element functor would store, the codes
// written once at the end. Handles every code, NaN and Inf included.
template <typename T, int OP>
__device__ __forceinline__ u32x4 fp8PackF32(const Red<T, OP>& fn, int n, const char* const* src, uint64_t i) {
  constexpr bool E5 = IsFp8<T>::e5m2;
  u32x4 cur = __builtin_nontemporal_load((const u32x4*)src[0] + i), nxt = cur;
  float acc[16];
  for (int k = 0; k < n; k++) {
    if (k + 1 < n) nxt = __builtin_nontemporal_load((const u32x4*)src[k + 1] + i);
    float x[16];
#pragma unroll
    for (int w = 0; w < 4; w++) fp8Decode4<E5>(cur[w], x + 4 * w);
    if constexpr (OP == DEV_PREMULSUM) {  // pre(x) = fromF(x * s), rounded like the functor
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        x[e] = opaqueF(x[e] * fn.s);
        x[e + 1] = opaqueF(x[e + 1] * fn.s);
        fp8RoundF<E5>(x[e], x[e + 1]);
      }
    }
    if (k == 0) {
#pragma unroll
      for (int e = 0; e < 16; e++) acc[e] = x[e];
    } else {
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        float r0, r1;
        if (OP == DEV_PROD) {
          r0 = opaqueF(x[e] * acc[e]);
          r1 = opaqueF(x[e + 1] * acc[e + 1]);
        } else if (OP == DEV_MINMAX) {
          r0 = fn.isMin ? minOrdered(x[e], acc[e]) : maxOrdered(x[e], acc[e]);
          r1 = fn.isMin ? minOrdered(x[e + 1], acc[e + 1]) : maxOrdered(x[e + 1], acc[e + 1]);
        } else {
          r0 = x[e] + acc[e];
          r1 = x[e + 1] + acc[e + 1];
        }
        fp8RoundF<E5>(r0, r1);
        acc[e] = r0;
        acc[e + 1] = r1;
      }
    }
    cur = nxt;
  }
  u32x4 out;
#pragma unroll
  for (int w = 0; w < 4; w++) out[w] = fp8Encode4<E5>(acc + 4 * w);
  return out;
}

// fp8 fold over 16-byte packs (the fp8 fold is ALU-bound: profiles/r03_dtype_rates_n2_onegpu.json). Default: the
// packed-half path (numerics.h fp8DecodeH2 / fp8RoundH2 / fp8EncodeH2x2) — the reference's half arithmetic two
// lanes per instruction, the accumulator as eight half pairs, one paired encode + decode per hop and lane pair;
// a pack with a NaN / Inf code in any source is recomputed by fp8PackF32 (NCCL_AMD_FP8_H2=0: always). One pack per
// thread per batch, the next source's pack in flight; 16-byte aligned ranges only (the < 16-byte tail per element).
#ifndef NCCL_AMD_FP8_H2
#define NCCL_AMD_FP8_H2 1
#endif
template <typename T, int OP>
__device__ __forceinline__ void foldFp8Packs(const Red<T, OP>& fn, int n, const char* const* src, uint64_t nelem,
                                             char* dstLocal, char* const* dstPush, int nPush) {
  constexpr bool E5 = IsFp8<T>::e5m2;
  const uint64_t npk = nelem / 16;
  const _Float16 sh = (_Float16)fn.s;  // PreMulSum scalar: an fp8 value, exact in half
  const fp8h2 s2 = {sh, sh};
  // a NaN / Inf scalar (a user PreMulSum op) can make NaN from finite codes: the f32 path then takes every pack
  const uint32_t scalarSpecial = (OP == DEV_PREMULSUM && !(__builtin_fabsf(fn.s) <= 65504.0f)) ? 1u : 0u;
  for (uint64_t i = threadIdx.x; i < npk; i += kThreads) {
    u32x4 out;
    if (NCCL_AMD_FP8_H2) {
      u32x4 cur = __builtin_nontemporal_load((const u32x4*)src[0] + i), nxt = cur;
      fp8h2 acc[8];
      uint32_t special = scalarSpecial;
      for (int k = 0; k < n; k++) {
        if (k + 1 < n) nxt = __builtin_nontemporal_load((const u32x4*)src[k + 1] + i);
        special |= fp8Special<E5>(cur[0]) | fp8Special<E5>(cur[1]) | fp8Special<E5>(cur[2]) | fp8Special<E5>(cur[3]);
        fp8h2 x[8];
#pragma unroll
        for (int w = 0; w < 4; w++) {
          x[2 * w] = fp8DecodeH2<E5>(cur[w], false);
          x[2 * w + 1] = fp8DecodeH2<E5>(cur[w], true);
        }
        if constexpr (OP == DEV_PREMULSUM) {  // pre(x) = fromF(__hmul(x, s))
#pragma unroll
          for (int j = 0; j < 8; j++) x[j] = fp8RoundH2<E5>(x[j] * s2);
        }
        if (k == 0) {
#pragma unroll
          for (int j = 0; j < 8; j++) acc[j] = x[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; j++) {
            if (OP == DEV_MINMAX)  // finite values: IEEE minimum / maximum order -0 below +0, like minOrdered
              acc[j] = fn.isMin ? __builtin_elementwise_minimum(x[j], acc[j]) : __builtin_elementwise_maximum(x[j], acc[j]);
            else if (OP == DEV_PROD)
              acc[j] = fp8RoundH2<E5>(x[j] * acc[j]);
            else
              acc[j] = fp8RoundH2<E5>(x[j] + acc[j]);
          }
        }
        cur = nxt;
      }
#pragma unroll
      for (int w = 0; w < 4; w++) out[w] = fp8EncodeH2x2<E5>(acc[2 * w], acc[2 * w + 1]);
      if (__builtin_expect(special != 0, 0)) out = fp8PackF32<T, OP>(fn, n, src, i);
    } else {
      out = fp8PackF32<T, OP>(fn, n, src, i);
    }
    if (dstLocal) __builtin_nontemporal_store(out, (u32x4*)dstLocal + i);
    for (int p = 0; p < nPush; p++) storeRemoteAt(remoteRsrc((u32x4*)dstPush[p] + (i - threadIdx.x)), threadIdx.x * 16u, out);
  }
  const uint64_t t = npk * 16 + threadIdx.x;  // < 16-byte tail
  if (t < nelem) {
    T a = fn.pre(((const T*)src[0])[t]);
    for (int k = 1; k < n; k++) a = fn.red(fn.pre(((const T*)src[k])[t]), a);
    a = fn.post(a);
    if (dstLocal) ((T*)dstLocal)[t] = a;
    for (int p = 0; p < nPush; p++) storeRemoteElt((T*)dstPush[p] + t, a);
  }
}

// Fold n sources into dst (and optionally into nPush remote copies). src[k] is the k-th source in
// fold order: acc = pre(src[0]); acc = red(pre(src[k]), acc) ...; out = post(acc).
// Source/destination pointer lists live in LDS (uniform, read by broadcast). Each thread owns U packs
// per batch and walks the sources with the next source's loads in flight while it reduces the
// current one (U*16 B x 2 per lane outstanding), so memory parallelism does not depend on n and the
// per-source loop needs no predication.
template <typename T, int OP, int UMAX = 64>
__device__ __forceinline__ void foldRange(const Red<T, OP>& fn, int n, const char* const* src, uint64_t nelem,
                                          char* dstLocal, char* const* dstPush, int nPush, bool aligned) {
  constexpr int EPP = 16 / sizeof(T);
  // uint8 / int8 Sum and MinMax fold four bytes per dword (numerics.h Swar8) and keep 2 packs in flight
  // (4 reach the 128-VGPR cap and spill in MinMax); other 1-byte folds (fp8, Prod, PreMulSum, integer avg) unpack 16 elements per pack into
  // separate registers, so they keep one pack per batch to stay within the register budget (kCoResident;
  // two packs spilled up to 55 VGPRs for fp8)
  // (integer avg on 1-byte types: the Sum fold on four bytes per dword, then numerics.h swarDivBytes)
  constexpr bool kSwarDiv = std::is_same<T, uint8_t>::value && OP == DEV_SUMPOSTDIV;
  constexpr bool kSwar = std::is_same<T, uint8_t>::value && (Swar8<OP>::ok || kSwarDiv);
  constexpr int kSwarOp = kSwarDiv ? DEV_SUM : OP;
  constexpr int U0 = sizeof(T) > 1 ? kFoldUnroll : kSwar ? kFoldUnrollSwar : kFoldUnroll1B;
  constexpr int U = U0 < UMAX ? U0 : UMAX;
  uint32_t swarMask = 0, divMagic = 0;
  if constexpr (kSwar && !kSwarDiv) swarMask = (uint32_t)(uint8_t)fn.arg * 0x01010101u;
  if constexpr (kSwarDiv) divMagic = swarDivMagic(fn.divisor);
  if constexpr (IsFp8<T>::value && NCCL_AMD_HW_FP8) {
    if (aligned) {
      foldFp8Packs<T, OP>(fn, n, src, nelem, dstLocal, dstPush, nPush);
      return;
    }
  }
  if (aligned) {
    const uint64_t npk = nelem / EPP;
    const uint64_t step = (uint64_t)U * kThreads;
    // (not for 1-byte types: their unpacked folds sit at the 128-VGPR cap, and the early loads spill there)
    constexpr bool kPrefetch = NCCL_AMD_FOLD_PREFETCH && sizeof(T) > 1;
    PackU<T> acc[U], cur[U], nxt[U];
    if constexpr (kPrefetch) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t i = threadIdx.x + (uint64_t)u * kThreads;
        if (i < npk) cur[u].v = __builtin_nontemporal_load((const u32x4*)src[0] + i);
      }
    }
    for (uint64_t base = threadIdx.x; base < npk; base += step) {
      if constexpr (!kPrefetch) {  // round 5's order: each batch starts by loading its first source
#pragma unroll
        for (int u = 0; u < U; u++) {
          uint64_t i = base + (uint64_t)u * kThreads;
          if (i < npk) cur[u].v = __builtin_nontemporal_load((const u32x4*)src[0] + i);
        }
      }
      for (int k = 0; k < n; k++) {
        // the next source's packs in flight while this one folds; after the last source, the NEXT batch's first
        // source (NCCL_AMD_FOLD_PREFETCH): the loads never drain between batches, which matters most at n = 2
        // (half of each batch had nothing in flight) and for remote sources (zero-copy kernels reading peers)
        const bool last = k + 1 == n;
        if (!last || (kPrefetch && base + step < npk)) {
          const u32x4* s = (const u32x4*)src[last ? 0 : k + 1];
          const uint64_t b = last ? base + step : base;
#pragma unroll
          for (int u = 0; u < U; u++) {
            uint64_t i = b + (uint64_t)u * kThreads;
            if (i < npk) nxt[u].v = __builtin_nontemporal_load(s + i);
          }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          if constexpr (kSwar) {
#pragma unroll
            for (int w = 0; w < 4; w++) acc[u].v[w] = k == 0 ? cur[u].v[w] : Swar8<kSwarOp>::red(cur[u].v[w], acc[u].v[w], swarMask);
          } else {
#pragma unroll
            for (int e = 0; e < EPP; e++) {
              T x = fn.pre(cur[u].e[e]);
              acc[u].e[e] = k == 0 ? x : fn.red(x, acc[u].e[e]);
            }
            // 1-byte types: keep the accumulator packed between sources (4 registers, not 16 unpacked bytes)
            if constexpr (sizeof(T) == 1 && NCCL_AMD_FOLD_REPACK) asm volatile("" : "+v"(acc[u].v));
          }
          cur[u] = nxt[u];
        }
      }
      LocalStore ls(dstLocal, base - threadIdx.x);
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t i = base + (uint64_t)u * kThreads;
        if (i >= npk) continue;
        if constexpr (kSwarDiv) {
#pragma unroll
          for (int w = 0; w < 4; w++) acc[u].v[w] = swarDivBytes(acc[u].v[w], divMagic, fn.isSigned);
        } else {
#pragma unroll
          for (int e = 0; e < EPP; e++) acc[u].e[e] = fn.post(acc[u].e[e]);
        }
        if (dstLocal) ls.put(threadIdx.x + u * kThreads, acc[u].v);
        for (int p = 0; p < nPush; p++) {
          // resource rebased on the batch's first pack: 32-bit offsets at any range size
          if (NCCL_AMD_BUFFER_STORES)
            storeRemoteAt(remoteRsrc((u32x4*)dstPush[p] + (base - threadIdx.x)), (threadIdx.x + u * kThreads) * 16u, acc[u].v);
          else storeRemote((u32x4*)dstPush[p] + i, acc[u].v);
        }
      }
    }
    const uint64_t t = npk * EPP + threadIdx.x;  // < 16-byte tail of the range
    if (t < nelem) {
      T acc = fn.pre(((const T*)src[0])[t]);
      for (int k = 1; k < n; k++) acc = fn.red(fn.pre(((const T*)src[k])[t]), acc);
      acc = fn.post(acc);
      if (dstLocal) ((T*)dstLocal)[t] = acc;
      for (int p = 0; p < nPush; p++) storeRemoteElt((T*)dstPush[p] + t, acc);
    }
  } else {
    for (uint64_t t = threadIdx.x; t < nelem; t += kThreads) {
      T acc = fn.pre(((const T*)src[0])[t]);
      for (int k = 1; k < n; k++) acc = fn.red(fn.pre(((const T*)src[k])[t]), acc);
      acc = fn.post(acc);
      if (dstLocal) ((T*)dstLocal)[t] = acc;
      for (int p = 0; p < nPush; p++) storeRemoteElt((T*)dstPush[p] + t, acc);
    }
  }
}


// ------------------------------------------------------------------------------------ collective kernel

// COLL_AR1 = one-shot AllReduce for small buffers: every rank publishes its whole channel portion to
// every peer and folds all n contributions itself (one handshake instead of three; (n-1)*S link bytes
// instead of 2(n-1)/n*S). Same fold order as the two-shot path, so results are identical.
// COLL_ARREF = the direct AllReduce on the reference's ring partition (NCCL_AMD_REF_ORDER, Channel::refPart): its
// own instantiation, so the default AllReduce kernel carries none of its indexing.
enum Coll { COLL_AR = 0, COLL_RS = 1, COLL_AG = 2, COLL_REDUCE = 3, COLL_AR1 = 4, COLL_ARREF = 5 };

// Element range [lo,hi) of a block handled by channel c at pipeline step s (offsets inside the block).
__device__ __forceinline__ void sliceRange(const CollArgs& a, int c, int s, uint64_t blockLen, uint64_t& lo,
                                           uint64_t& hi) {
  uint64_t pEnd = min((uint64_t)(c + 1) * a.part, blockLen);
  lo = min((uint64_t)c * a.part + (uint64_t)s * a.slice, pEnd);
  hi = min(lo + a.slice, pEnd);
}

// COLL_ARREF channel geometry (Channel::refInit): region offset, loop length, full loops, the last loop's length
// and chunk, this workgroup's sub-chunk length in a full / the last loop, steps per full loop, steps in all, and
// which sub-chunk of every chunk this workgroup moves.
struct RefGeom {
  uint64_t off, loop, rem, ckLast, scFull, scLast;
  uint32_t full, perFull, steps, sub;
};
// Per-workgroup (channel) LDS scratch for the handshake arrays.
struct Shared {
  ChanState st;
  WaitProbe probe;  // staged waits: a peer's SYM_ENTER beyond this channel's symmetric epoch is a mismatch
  RefGeom ref;
  const char* srcPtr[NCCL_AMD_MAX_RANKS];   // phase-B fold sources, in fold order
  char* pushPtr[NCCL_AMD_MAX_RANKS];        // phase-B remote destinations
  int nPush;
  uint64_t want[NCCL_AMD_MAX_RANKS];
  uint64_t* sigPtr[2 * NCCL_AMD_MAX_RANKS];
  uint64_t sigVal[2 * NCCL_AMD_MAX_RANKS];
};

template <typename T, int OP, int COLL>
struct Channel {
  const CollArgs& a;
  const DevComm& dc;
  Shared& sh;
  const Red<T, OP>& fn;
  int c, me, n, nSlots;
  bool aligned, isRoot, forceAcq, forceRel, noRel, noAcq;
  // AG pull (NCCL_AMD_AG_PULL=1, AllReduce / AllGather): phase B leaves ONE copy of the owner's block in
  // its own AG staging and phase C reads it from there over xGMI, instead of B pushing n-1 copies into
  // the peers' staging. Same link bytes, reads instead of writes. The copy is shared by all readers, so
  // it runs on its own per-channel sequence (CTR_PULL_PUB / CTR_PULL_GOT, FLG_PULL_READY / FLG_PULL_ACK):
  // the slot is reused only after EVERY peer acked, and the per-pair AG counters (which a Reduce, pushing
  // to its root only, advances unevenly) are left alone.
  bool agPull;
  // RS pull (NCCL_AMD_RS_PULL=1, AllReduce / ReduceScatter): phase A copies my input's block-p slice into
  // MY OWN RS staging (area "for p", a local copy) and owner p's fold reads it from there over xGMI,
  // instead of A writing it into p's staging. Same link bytes as reads; slots, credits and flags unchanged.
  bool rsPull;
  // the op's own channel index, which cuts its data (sliceRange); c is the physical channel (workgroup)
  // whose staging, flags and credits carry it. They differ only inside a group batch (collBatchKernel).
  int cl;
  static constexpr uint64_t ts = sizeof(T);
  static constexpr bool kAR = COLL == COLL_AR || COLL == COLL_ARREF;

  __device__ uint64_t blockLen(int q) const {
    if (kAR || COLL == COLL_REDUCE) {
      uint64_t b = (uint64_t)q * a.chunk;
      return b >= a.count ? 0 : min(a.chunk, a.count - b);
    }
    return a.chunk;
  }
  __device__ uint64_t& ctr(int k, int r) const { return sh.st.ctr[k][r]; }
  // NCCL_AMD_REF_ORDER (COLL_ARREF): the reference's ring partition instead of rank blocks cut into
  // channel parts. This channel walks its part (ncclCollCbdPart, device.h:337-361: cbdLo / part / cbdHi) in loops
  // of n chunks of a.chunk elements, the last loop's chunk re-cut to alignUp(divUp(rem, n), 16 / sizeof(T))
  // (all_reduce.h:34-38); chunk q of a loop is "block" q, owned and finalised by rank q, so every element folds
  // q+1, ..., q as in the reference's ring. a.refSub workgroups share one reference part: workgroup cl serves part
  // cl / refSub and moves sub-chunk cl % refSub (alignUp(divUp(chunk, refSub), 16 / sizeof(T)) elements) of every
  // chunk of it — which workgroup moves an element never changes its fold order, so the reference's channel count
  // and the launch's parallelism are independent. Step s = slice j of the sub-chunk of loop l.
  static constexpr bool refPart() { return COLL == COLL_ARREF; }
  // this channel's region and loop geometry, computed once per launch (refInit) into LDS (Shared::ref): the 64-bit
  // divisions stay out of the per-step code and the values out of the registers the fold needs
  __device__ void refInit() {
    constexpr uint64_t EPP = 16 / sizeof(T);
    if (threadIdx.x == 0) {
      const uint32_t G = a.refSub;
      const int nParts = (int)(gridDim.x / G);  // never batched: the grid is the op's channels
      const int k = (int)((uint32_t)cl / G);
      uint64_t off, cnt;
      if (k == 0) off = 0, cnt = a.cbdLo;
      else if (k == nParts - 1) off = a.cbdLo + (uint64_t)(nParts - 2) * a.part, cnt = a.cbdHi;
      else off = a.cbdLo + (uint64_t)(k - 1) * a.part, cnt = a.part;
      RefGeom& g = sh.ref;
      g.off = off;
      g.sub = (uint32_t)cl - (uint32_t)k * G;
      g.loop = (uint64_t)n * a.chunk;
      g.full = (uint32_t)(cnt / g.loop);
      g.rem = cnt - (uint64_t)g.full * g.loop;
      g.ckLast = g.rem ? ((g.rem + n - 1) / n + EPP - 1) / EPP * EPP : 0;
      g.scFull = ((a.chunk + G - 1) / G + EPP - 1) / EPP * EPP;
      g.scLast = ((g.ckLast + G - 1) / G + EPP - 1) / EPP * EPP;
      // this sub-chunk's length in a chunk of length ck (block 0's, the longest of a loop)
      auto subLen = [&](uint64_t ck, uint64_t sc) -> uint64_t {
        const uint64_t lo = min((uint64_t)g.sub * sc, ck);
        return min(lo + sc, ck) - lo;
      };
      g.perFull = (uint32_t)((subLen(a.chunk, g.scFull) + a.slice - 1) / a.slice);
      g.steps = g.full * g.perFull + (uint32_t)((subLen(g.ckLast, g.scLast) + a.slice - 1) / a.slice);
    }
    __syncthreads();
  }
  // Block b's slice at pipeline step `step`: elements [off, off + len) of the buffer.
  __device__ void blockSlice(int step, int b, uint64_t& off, uint64_t& len) const {
    uint64_t lo, hi;
    if (!refPart()) {
      sliceRange(a, cl, step, blockLen(b), lo, hi);
      off = (uint64_t)b * a.chunk + lo;
      len = hi - lo;
      return;
    }
    const RefGeom& g = sh.ref;
    const uint32_t st = (uint32_t)step, inFull = g.full * g.perFull;
    uint32_t l, j;
    uint64_t ck, rem, sc;
    if (st < inFull) l = st / g.perFull, j = st - l * g.perFull, ck = a.chunk, rem = g.loop, sc = g.scFull;
    else l = g.full, j = st - inFull, ck = g.ckLast, rem = g.rem, sc = g.scLast;
    const uint64_t bb = (uint64_t)b * ck, blen = bb >= rem ? 0 : min(ck, rem - bb);
    const uint64_t sLo = min((uint64_t)g.sub * sc, blen), sHi = min(sLo + sc, blen);  // my sub-chunk of block b
    lo = min(sLo + (uint64_t)j * a.slice, sHi);
    hi = min(lo + a.slice, sHi);
    off = g.off + (uint64_t)l * g.loop + bb + lo;
    len = hi - lo;
  }
  // k-th peer (k = 1..n-1) this channel sends to (scatter) or reads from (pull gather), staggered by channel
  // (chanPeer, device_abi.h): all of a rank's channels on ONE xGMI link at a time otherwise.
  __device__ int peerAt(int k) const { return chanPeer(me, n, c, k); }
  __device__ const uint64_t* myFlags(int kind) const { return dc.flags[me] + flagIndex(c, kind, 0); }
  __device__ bool pushesTo(int p) const {
    if (kAR || COLL == COLL_AG) return true;
    return COLL == COLL_REDUCE && !isRoot && p == a.root;
  }
  // Reduce over n >= 3 ranks: the root owns no block — the buffer is cut into n-1 blocks owned by the other
  // ranks — so the root's links carry only the n-1 reduced blocks in (S in total) instead of its own
  // block's n-1 contributions plus the n-1 reduced blocks (2(n-1)/n * S). Fold order is unchanged
  // (root+1, ..., root, reduce.h:34-52): it never depended on who folds.
  __device__ bool rootless() const { return COLL == COLL_REDUCE && n >= 3; }
  __device__ bool owns(int r) const { return !rootless() || r != a.root; }
  __device__ int blockOf(int r) const { return rootless() && r > a.root ? r - 1 : r; }

  // A: scatter input block p to owner p's RS staging (AR, RS, REDUCE)
  __device__ bool phaseA(int step) {
    int tid = threadIdx.x;
    if (tid < NCCL_AMD_MAX_RANKS) {
      uint64_t s = ctr(CTR_SEND_RS, tid);
      sh.want[tid] = (tid < n && tid != me && owns(tid) && s + 1 > (uint64_t)nSlots) ? s + 1 - nSlots : 0;
    }
    __syncthreads();
    if (!waitAll(dc, sh.st, myFlags(FLG_RS_ACK), sh.want, forceAcq)) return false;
    for (int k = 1; k < n; k++) {
      int p = peerAt(k);
      if (!owns(p)) continue;
      const int b = blockOf(p);
      uint64_t off, len;
      blockSlice(step, b, off, len);
      int slot = (int)(ctr(CTR_SEND_RS, p) % nSlots);
      char* dst = rsPull ? dc.staging[me] + stagingOffset(dc, c, STG_RS, slot, p)   // my slab, area for p
                         : dc.staging[p] + stagingOffset(dc, c, STG_RS, slot, me);
      const char* src = (const char*)a.sendbuff + off * ts;
      copyRange<T, true>(dst, src, len * ts, aligned);
    }
    if (tid < NCCL_AMD_MAX_RANKS) {
      bool act = tid < n && tid != me && owns(tid);
      sh.sigVal[tid] = act ? ctr(CTR_SEND_RS, tid) + 1 : 0;
      sh.sigPtr[tid] = act ? dc.flags[tid] + flagIndex(c, FLG_RS_READY, me) : nullptr;
    }
    __syncthreads();
    signalAll(sh.sigPtr, sh.sigVal, NCCL_AMD_MAX_RANKS, !noRel);
    if (tid < n && tid != me && owns(tid)) ctr(CTR_SEND_RS, tid)++;
    __syncthreads();
    return true;
  }

  // B: fold my block (AR, RS, REDUCE) or publish my input block (AG); push to AG staging
  __device__ bool phaseB(int step) {
    if (rootless() && isRoot) return true;  // the root owns no block
    int tid = threadIdx.x;
    const bool push = (kAR || COLL == COLL_AG || (COLL == COLL_REDUCE && !isRoot));
    if (COLL != COLL_AG) {
      if (tid < NCCL_AMD_MAX_RANKS) sh.want[tid] = (tid < n && tid != me) ? ctr(CTR_RECV_RS, tid) + 1 : 0;
      __syncthreads();
      if (!waitAll<PROBE_STAGED>(dc, sh.st, myFlags(FLG_RS_READY), sh.want, !noAcq, &sh.probe)) return false;
    }
    if (push) {
      if (tid < NCCL_AMD_MAX_RANKS) {
        // pull: slot pub % nSlots is free once EVERY peer acked publication pub - nSlots
        uint64_t s = agPull ? ctr(CTR_PULL_PUB, 0) : ctr(CTR_SEND_AG, tid);
        bool dstPeer = tid < n && tid != me && pushesTo(tid);
        sh.want[tid] = (dstPeer && s + 1 > (uint64_t)nSlots) ? s + 1 - nSlots : 0;
      }
      __syncthreads();
      if (!waitAll(dc, sh.st, myFlags(agPull ? FLG_PULL_ACK : FLG_AG_ACK), sh.want, forceAcq)) return false;
    }
    const int myB = blockOf(me);
    uint64_t lo, hi;
    sliceRange(a, cl, step, blockLen(myB), lo, hi);
    uint64_t myOff = (uint64_t)myB * a.chunk + lo, nelem = hi - lo;  // my block's slice in the buffer
    if (refPart()) blockSlice(step, myB, myOff, nelem);
    if (tid == 0) {
      int np = 0;
      if (agPull) {  // one copy in my own AG staging, at this channel's publication sequence
        sh.pushPtr[np++] = dc.staging[me] + stagingOffset(dc, c, STG_AG, (int)(ctr(CTR_PULL_PUB, 0) % nSlots), me);
      } else {
        for (int k = 1; k < n; k++) {
          int p = (me + k) % n;
          if (pushesTo(p))
            sh.pushPtr[np++] = dc.staging[p] + stagingOffset(dc, c, STG_AG, (int)(ctr(CTR_SEND_AG, p) % nSlots), me);
        }
      }
      sh.nPush = np;
      // fold order: owner+1, ..., owner (AR/RS, all_reduce.h:43-66) or root+1, ..., root (reduce.h:34-52)
      int first = (COLL == COLL_REDUCE ? a.root + 1 : me + 1) % n;
      for (int k = 0; k < n; k++) {
        int q = (first + k) % n;
        const int rslot = (int)(ctr(CTR_RECV_RS, q) % nSlots);
        sh.srcPtr[k] = q == me ? (const char*)a.sendbuff + myOff * ts
                     : rsPull  ? dc.staging[q] + stagingOffset(dc, c, STG_RS, rslot, me)  // q's slab, remote
                               : dc.staging[me] + stagingOffset(dc, c, STG_RS, rslot, q);
      }
    }
    __syncthreads();
    if (COLL == COLL_AG) {
      const char* src = (const char*)a.sendbuff + lo * ts;
      char* dst = (char*)a.recvbuff + ((uint64_t)me * a.chunk + lo) * ts;
      copyRangeMulti<T>(dst != src ? dst : nullptr, sh.pushPtr, sh.nPush, src, nelem * ts, aligned);
    } else {
      char* dstLocal = nullptr;
      if (COLL == COLL_RS) dstLocal = (char*)a.recvbuff + lo * ts;
      else if (kAR || isRoot) dstLocal = (char*)a.recvbuff + myOff * ts;
      // (the reference-order kernel's extra indexing leaves the widest folds — 1-byte unpacked, 8-byte — fewer
      // packs in flight within the 128-VGPR co-residency budget)
      constexpr int kUMax = COLL != COLL_ARREF ? 64 : sizeof(T) == 1 ? 1 : sizeof(T) == 8 ? 2 : 64;
      foldRange<T, OP, kUMax>(fn, n, sh.srcPtr, nelem, dstLocal, sh.pushPtr, sh.nPush, aligned);
    }
    // one release covers both: AG data ready at each destination; RS slots consumed (ack to senders)
    if (tid < NCCL_AMD_MAX_RANKS) {
      bool peer = tid < n && tid != me;
      bool dstPeer = peer && push && pushesTo(tid);
      sh.sigVal[tid] = dstPeer ? (agPull ? ctr(CTR_PULL_PUB, 0) : ctr(CTR_SEND_AG, tid)) + 1 : 0;
      sh.sigPtr[tid] = dstPeer ? dc.flags[tid] + flagIndex(c, agPull ? FLG_PULL_READY : FLG_AG_READY, me) : nullptr;
      bool ack = peer && COLL != COLL_AG;
      sh.sigVal[NCCL_AMD_MAX_RANKS + tid] = ack ? ctr(CTR_RECV_RS, tid) + 1 : 0;
      sh.sigPtr[NCCL_AMD_MAX_RANKS + tid] = ack ? dc.flags[tid] + flagIndex(c, FLG_RS_ACK, me) : nullptr;
    }
    __syncthreads();
    signalAll(sh.sigPtr, sh.sigVal, 2 * NCCL_AMD_MAX_RANKS, (push && !noRel) || forceRel);
    if (tid < n && tid != me) {
      if (COLL != COLL_AG) ctr(CTR_RECV_RS, tid)++;
      if (push && pushesTo(tid) && !agPull) ctr(CTR_SEND_AG, tid)++;
    }
    if (agPull && tid == 0) ctr(CTR_PULL_PUB, 0)++;
    __syncthreads();
    return true;
  }

  // One-shot A: publish my portion [lo,hi) of the whole buffer to every peer's RS staging.
  __device__ bool oneShotA(int step) {
    int tid = threadIdx.x;
    if (tid < NCCL_AMD_MAX_RANKS) {
      uint64_t s = ctr(CTR_SEND_RS, tid);
      sh.want[tid] = (tid < n && tid != me && s + 1 > (uint64_t)nSlots) ? s + 1 - nSlots : 0;
    }
    __syncthreads();
    if (!waitAll(dc, sh.st, myFlags(FLG_RS_ACK), sh.want, forceAcq)) return false;
    uint64_t lo, hi;
    sliceRange(a, cl, step, a.count, lo, hi);
    const char* src = (const char*)a.sendbuff + lo * ts;
    if (threadIdx.x == 0) {
      for (int k = 1; k < n; k++) {
        int p = peerAt(k);
        sh.pushPtr[k - 1] = dc.staging[p] + stagingOffset(dc, c, STG_RS, (int)(ctr(CTR_SEND_RS, p) % nSlots), me);
      }
    }
    __syncthreads();
    copyRangeMulti<T>(nullptr, sh.pushPtr, n - 1, src, (hi - lo) * ts, aligned);
    if (tid < NCCL_AMD_MAX_RANKS) {
      bool act = tid < n && tid != me;
      sh.sigVal[tid] = act ? ctr(CTR_SEND_RS, tid) + 1 : 0;
      sh.sigPtr[tid] = act ? dc.flags[tid] + flagIndex(c, FLG_RS_READY, me) : nullptr;
    }
    __syncthreads();
    signalAll(sh.sigPtr, sh.sigVal, NCCL_AMD_MAX_RANKS, !noRel);
    if (tid < n && tid != me) ctr(CTR_SEND_RS, tid)++;
    __syncthreads();
    return true;
  }

  // One-shot B: fold all n contributions of my portion, owner by owner (the portion may straddle
  // rank blocks; block q folds q+1, ..., q like the two-shot path), then return the credits.
  __device__ bool oneShotB(int step) {
    int tid = threadIdx.x;
    if (tid < NCCL_AMD_MAX_RANKS) sh.want[tid] = (tid < n && tid != me) ? ctr(CTR_RECV_RS, tid) + 1 : 0;
    __syncthreads();
    if (!waitAll<PROBE_STAGED>(dc, sh.st, myFlags(FLG_RS_READY), sh.want, !noAcq, &sh.probe)) return false;
    uint64_t lo, hi;
    sliceRange(a, cl, step, a.count, lo, hi);
    for (uint64_t x = lo; x < hi;) {
      const int owner = (int)(x / a.chunk);
      const uint64_t end = min(hi, (uint64_t)(owner + 1) * a.chunk);
      if (tid == 0) {
        int first = (owner + 1) % n;
        for (int k = 0; k < n; k++) {
          int q = (first + k) % n;
          sh.srcPtr[k] = q == me ? (const char*)a.sendbuff + x * ts
                                 : dc.staging[me] + stagingOffset(dc, c, STG_RS, (int)(ctr(CTR_RECV_RS, q) % nSlots), q) +
                                       (x - lo) * ts;
        }
      }
      __syncthreads();
      // sub-range starts inside a slot are 16-byte aligned: rank blocks are multiples of 16 bytes
      foldRange<T, OP>(fn, n, sh.srcPtr, end - x, (char*)a.recvbuff + x * ts, sh.pushPtr, 0, aligned);
      __syncthreads();
      x = end;
    }
    if (tid < NCCL_AMD_MAX_RANKS) {
      bool peer = tid < n && tid != me;
      sh.sigVal[tid] = peer ? ctr(CTR_RECV_RS, tid) + 1 : 0;
      sh.sigPtr[tid] = peer ? dc.flags[tid] + flagIndex(c, FLG_RS_ACK, me) : nullptr;
    }
    __syncthreads();
    signalAll(sh.sigPtr, sh.sigVal, NCCL_AMD_MAX_RANKS, forceRel);  // credits only
    if (tid < n && tid != me) ctr(CTR_RECV_RS, tid)++;
    __syncthreads();
    return true;
  }

  // C: gather the other blocks from my AG staging into the output (AR, AG, REDUCE at root)
  __device__ bool phaseC(int step) {
    int tid = threadIdx.x;
    const int recvKind = agPull ? CTR_PULL_GOT : CTR_RECV_AG;
    if (tid < NCCL_AMD_MAX_RANKS) sh.want[tid] = (tid < n && tid != me) ? ctr(recvKind, tid) + 1 : 0;
    __syncthreads();
    if (!waitAll<PROBE_STAGED>(dc, sh.st, myFlags(agPull ? FLG_PULL_READY : FLG_AG_READY), sh.want, !noAcq, &sh.probe)) return false;
    // peers in the channel-rotated order: copyRange is workgroup-wide, so one order on every
    // channel would pull from one owner at a time — one incoming link of n-1 — while all channels move in step
    for (int k = 1; k < n; k++) {
      const int q = peerAt(k);
      const int b = blockOf(q);  // the block rank q owns (its index shifts past the root when rootless)
      uint64_t off, len;
      blockSlice(step, b, off, len);
      const int slot = (int)(ctr(recvKind, q) % nSlots);
      const char* src = agPull ? dc.staging[q] + stagingOffset(dc, c, STG_AG, slot, q)  // q's own copy, remote
                               : dc.staging[me] + stagingOffset(dc, c, STG_AG, slot, q);
      char* dst = (char*)a.recvbuff + off * ts;
      copyRange<T, false>(dst, src, len * ts, aligned);
    }
    if (tid < NCCL_AMD_MAX_RANKS) {
      bool peer = tid < n && tid != me;
      sh.sigVal[tid] = peer ? ctr(recvKind, tid) + 1 : 0;
      sh.sigPtr[tid] = peer ? dc.flags[tid] + flagIndex(c, agPull ? FLG_PULL_ACK : FLG_AG_ACK, me) : nullptr;
    }
    __syncthreads();
    signalAll(sh.sigPtr, sh.sigVal, NCCL_AMD_MAX_RANKS, forceRel);  // credits only
    if (tid < n && tid != me) ctr(recvKind, tid)++;
    __syncthreads();
    return true;
  }
};

// Per-channel credit counters live in device memory between launches; a workgroup keeps them in LDS.
__device__ __forceinline__ void loadCounters(const DevComm& dc, Shared& sh, int c) {
  const int tid = threadIdx.x;
  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    sh.st.ctr[k][r] = dc.counters[ctrIndex(c, k, r)];
  }
  if (tid == 0) {
    sh.st.abort = 0;
    sh.probe.flag[0] = dc.flags[dc.rank] + flagIndex(c, FLG_SYM_ENTER, 0);
    sh.probe.epoch = dc.counters[ctrIndex(c, CTR_SYM, 0)];
  }
  __syncthreads();
}
__device__ __forceinline__ void storeCounters(const DevComm& dc, Shared& sh, int c) {
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    dc.counters[ctrIndex(c, k, r)] = sh.st.ctr[k][r];
  }
}
// The functor's scalar: ncclScalarDevice PreMulSum dereferences it at run time (reference onerank.cu:31-41).
template <typename T>
__device__ __forceinline__ uint64_t redArgOf(uint64_t arg, const void* ptr) {
  if (!ptr) return arg;
  uint64_t v = 0;
  __builtin_memcpy(&v, ptr, sizeof(T));
  return v;
}

// One op's logical channel cl on physical channel c. False once a wait timed out (the comm aborts).
template <typename T, int OP, int COLL>
__device__ __forceinline__ bool runChannel(const CollArgs& a, const DevComm& dc, Shared& sh, const Red<T, OP>& fn,
                                           int c, int cl) {
  // protoFlags: 1 = acquire on credit waits too, 2 = release on credit signals too, 4 = C(s) before A(s+1),
  // 8 = no release fence before data flags (the default: every published byte is a write-through system-scope
  // store drained before the flag; NCCL_AMD_P2P_FENCE=1 clears it), 16 = AG pull
  // (NCCL_AMD_AG_PULL=1), 32 = RS pull (NCCL_AMD_RS_PULL=1), 64 = no acquire after data waits (diagnostics
  // only: measures the acquire's cost)
  Channel<T, OP, COLL> ch{a, dc, sh, fn, c, dc.rank, dc.nRanks, dc.nSlots, a.aligned != 0,
                          (COLL != COLL_REDUCE) || dc.rank == a.root, (a.protoFlags & 1) != 0,
                          (a.protoFlags & 2) != 0, (a.protoFlags & 8) != 0, (a.protoFlags & 64) != 0,
                          (COLL == COLL_AR || COLL == COLL_ARREF || COLL == COLL_AG) && (a.protoFlags & 16) != 0,
                          (COLL == COLL_AR || COLL == COLL_ARREF || COLL == COLL_RS) && (a.protoFlags & 32) != 0, cl};
  if (COLL == COLL_AR1) {
    bool ok = true;
    for (int s = 0; ok && s < a.nSteps; s++) ok = ch.oneShotA(s) && ch.oneShotB(s);
    return ok;
  }
  constexpr bool hasA = COLL != COLL_AG;
  const bool hasC = COLL == COLL_AR || COLL == COLL_ARREF || COLL == COLL_AG || (COLL == COLL_REDUCE && ch.isRoot);
  // Pipeline: A(0); for s: B(s); A(s+1); C(s). Hoisting A(s+1) above C(s) lets the owners start
  // reducing step s+1 while this rank still drains step s (they are independent).
  if constexpr (Channel<T, OP, COLL>::refPart()) ch.refInit();
  const int nSteps = ch.refPart() ? (int)sh.ref.steps : a.nSteps;
  bool ok = !hasA || nSteps == 0 || ch.phaseA(0);
  const bool cFirst = (a.protoFlags & 4) != 0;
  for (int s = 0; ok && s < nSteps; s++) {
    ok = ch.phaseB(s);
    if (ok && hasC && cFirst) ok = ch.phaseC(s);
    if (ok && hasA && s + 1 < nSteps) ok = ch.phaseA(s + 1);
    if (ok && hasC && !cFirst) ok = ch.phaseC(s);
  }
  return ok;
}

template <typename T, int OP, int COLL>
__global__ void __launch_bounds__(kThreads) kCoResident collKernel(CollArgs a) {
  __shared__ Shared sh;
  const DevComm& dc = *a.comm;
  const int c = blockIdx.x;
  loadCounters(dc, sh, c);
  const Red<T, OP> fn(redArgOf<T>(a.redArg, a.redArgPtr));
  runChannel<T, OP, COLL>(a, dc, sh, fn, c, c);
  storeCounters(dc, sh, c);
}

// Group batch (reference: a group's ops aggregated into one kernel plan, enqueue.cc:405-470): up to
// kMaxCollBatch staged ops of one comm with the same collective, type and operator in ONE launch. Op k's
// channels are the physical channels chOff[k] .. chOff[k] + nch[k] - 1 (mod the grid), so consecutive ops run
// side by side on disjoint workgroups while the grid lasts and in op order on a shared one after that. Each
// rank forms the same batches with the same offsets, so every physical channel runs the same handshake
// sequence on every rank and its credits and slots carry over from op to op exactly as between launches.
template <typename T, int OP, int COLL>
__global__ void __launch_bounds__(kThreads) kCoResident collBatchKernel(CollBatchArgs b) {
  __shared__ Shared sh;
  __shared__ int chOffSh[kMaxCollBatch], nchSh[kMaxCollBatch];  // fetched in parallel (see llKernel)
  const DevComm& dc = *b.op[0].comm;
  const int c = blockIdx.x;
  if (threadIdx.x < (unsigned)b.nOps) {
    chOffSh[threadIdx.x] = b.chOff[threadIdx.x];
    nchSh[threadIdx.x] = b.nch[threadIdx.x];
  }
  loadCounters(dc, sh, c);  // (ends with a workgroup barrier)
  const Red<T, OP> fn(redArgOf<T>(b.op[0].redArg, b.op[0].redArgPtr));
  for (int k = 0; k < b.nOps; k++) {
    int j = c - chOffSh[k];
    if (j < 0) j += (int)gridDim.x;
    if (j >= nchSh[k]) continue;
    if (!runChannel<T, OP, COLL>(b.op[k], dc, sh, fn, c, j)) break;
  }
  storeCounters(dc, sh, c);
}

}  // namespace ncclamd
#include "pipe.h"  // ring and chain (NCCL_ALGO=RING / TREE) on the same staging and credits
namespace ncclamd {

// ------------------------------------------------------------------------------------ LL one-shot
//
// Low-latency AllReduce for small buffers (reference prims_ll.h:108-158, LL protocol). Every 8 bytes of
// payload travel as half of a 16-byte line {data32, flag32, data32, flag32} stored with ONE system-scope
// write-through store into each peer's LL area; the flag is the channel's LL epoch. A reader polls the
// lines themselves (8-byte system-scope atomic loads: each half is single-copy atomic), so neither side
// needs a flag word, a release fence or an acquire fence — the one-shot path's two handshakes and two
// cache-maintenance fences become one one-way trip. Line areas are double-buffered by epoch parity: a
// sender reaches epoch e+2 on a channel only after receiving every peer's e+1 lines, which each peer
// sends only after finishing epoch e, so parity e's lines are never overwritten while still unread.
// Fold order per element is the reference ring order of its owner block (owner+1, ..., owner): results
// are identical to the other AllReduce paths.
// A line is read with ONE 16-byte load (the reference's ld.volatile.v4, prims_ll.h): each 8-byte half {data32, flag32}
// is single-copy atomic, so a half whose flag matches carries its data whatever the other half shows. (Two 8-byte
// loads, the second issued only once the first had matched, put two memory latencies on every line of the poll.)
// The line area is uncached memory: no cached copy can be stale (loadLine16 / loadSeenLine16 below).
__device__ __forceinline__ uint64_t llPayload(u32x4 v) { return (uint64_t)v.x | ((uint64_t)v.z << 32); }
__device__ __forceinline__ u32x4 loadLine16(const char* p) { return *(const volatile u32x4*)p; }  // polls
// Re-reads of lines a poll has already seen complete: uncached memory, so a plain load cannot hit a stale
// copy; not volatile, so the loads of several peers' lines can be in flight together.
__device__ __forceinline__ u32x4 loadSeenLine16(const char* p) { return __builtin_nontemporal_load((const u32x4*)p); }

template <typename T, int OP>
__device__ __forceinline__ bool llChannelOp(const DevComm& dc, const Red<T, OP>& fn, const LLOp& op, int c, int j,
                                            uint64_t e64, int& abortSh) {
  // c: physical channel (line area + epoch); j: this op's part index on it. Payload space: AllReduce the
  // whole buffer; ReduceScatter / AllGather one rank block (rank p's line for payload pk carries block p's
  // payload pk for ReduceScatter, its own input's payload pk for AllGather).
  const int tid = threadIdx.x, me = dc.rank, n = dc.nRanks;
  constexpr int EPP = 8 / sizeof(T);  // elements per 8-byte payload
  const uint32_t flag = (uint32_t)e64 ? (uint32_t)e64 : 1u;  // never 0 (the area starts zeroed)
  const int par = (int)(e64 & 1);
  const uint64_t nbytes = op.count * sizeof(T);
  const uint64_t npk = (nbytes + 7) / 8;
  const uint64_t lo = min((uint64_t)j * op.part, npk), hi = min(lo + op.part, npk);
  const char* send = (const char*)op.send;
  char* recv = (char*)op.recv;
  // Payloads are 8 bytes of the user buffer at any alignment: the LL decision is rank-uniform (enqueue.cc
  // llPlan), so a buffer that is only 4-, 2- or 1-byte aligned on some rank still takes this path there.
  auto payload = [&](const char* base, uint64_t pk) -> uint64_t {
    const char* p = base + pk * 8;
    const uintptr_t al = (uintptr_t)p;
    uint64_t v = 0;
    if (pk * 8 + 8 <= nbytes) {
      if ((al & 7) == 0) v = *(const uint64_t*)p;
      else if ((al & 3) == 0) v = ((const uint32_t*)p)[0] | ((uint64_t)((const uint32_t*)p)[1] << 32);
      else for (int b = 0; b < 8; b++) v |= (uint64_t)(unsigned char)p[b] << (8 * b);
    } else {
      for (uint64_t b = pk * 8; b < nbytes; b++) v |= (uint64_t)(unsigned char)base[b] << (8 * (b - pk * 8));
    }
    return v;
  };
  auto storePayload = [&](char* base, uint64_t pk, uint64_t v) {
    char* p = base + pk * 8;
    const uintptr_t al = (uintptr_t)p;
    if (pk * 8 + 8 <= nbytes) {
      if ((al & 7) == 0) {
        *(uint64_t*)p = v;
      } else if ((al & 3) == 0) {
        ((uint32_t*)p)[0] = (uint32_t)v;
        ((uint32_t*)p)[1] = (uint32_t)(v >> 32);
      } else {
        for (int b = 0; b < 8; b++) p[b] = (char)(v >> (8 * b));
      }
    } else {
      for (uint64_t b = pk * 8; b < nbytes; b++) base[b] = (char)(v >> (8 * (b - pk * 8)));
    }
  };

  // send: payloads [lo,hi) to every peer, 16-byte lines (two 8-byte payloads per thread step)
  for (uint64_t i = lo + 2 * tid; i < hi; i += 2 * kThreads) {
    const uint64_t off = (i - lo) * 16;  // payload pk's line sits at (pk - lo) * 16
    uint64_t v0 = 0, v1 = 0;
    if (op.coll != LL_RS) {
      v0 = payload(send, i);
      if (i + 1 < hi) v1 = payload(send, i + 1);
    }
    for (int k = 1; k < n; k++) {
      int p = (me + k) % n;
      if (op.coll == LL_RS) {  // block p goes to its owner
        v0 = payload(send + (uint64_t)p * nbytes, i);
        if (i + 1 < hi) v1 = payload(send + (uint64_t)p * nbytes, i + 1);
      }
      char* base = (char*)dc.flags[p] + llLineOffset(dc, c, par, me) + off;
      storeRemote(base, u32x4{(uint32_t)v0, flag, (uint32_t)(v0 >> 32), flag});
      if (i + 1 < hi) storeRemote(base + 16, u32x4{(uint32_t)v1, flag, (uint32_t)(v1 >> 32), flag});
    }
  }
  // receive: one 8-byte payload per thread step (after the barrier every input byte has been sent, so an
  // in-place output cannot overwrite a payload another thread still has to send)
  __syncthreads();
  const uint64_t t0 = clockTicks();
  bool ok = true;
  const char* myLL = (const char*)dc.flags[me];
  const bool folds = op.coll != LL_AG && !(op.coll == LL_REDUCE && me != op.root);
  const char* mine = op.coll == LL_RS ? send + (uint64_t)me * nbytes : send;
  for (uint64_t pk = lo + tid; pk < hi; pk += kThreads) {
    // my own contribution, loaded before the wait so its latency hides behind the peers' lines
    const uint64_t myV = folds ? payload(mine, pk) : 0;
    // pass 1: wait until every peer's line for this payload carries this epoch's flag
    uint32_t pending = 0;
    for (int q = 0; q < n; q++)
      if (q != me) pending |= 1u << q;
    uint32_t spins = 0;
    while (pending) {
      for (int q = 0; q < n; q++) {
        if (!(pending & (1u << q))) continue;
        const u32x4 v = loadLine16(myLL + llLineOffset(dc, c, par, q) + (pk - lo) * 16);
        if (v.y == flag && v.w == flag) pending &= ~(1u << q);
      }
      if (pending) __builtin_amdgcn_s_sleep(1);
      if (pending && (++spins & 1023) == 0) {
        if (__hip_atomic_load(dc.abortFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          reportError(dc, DERR_ABORT);
          abortSh = 1;
        } else if (__hip_atomic_load(dc.errorWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                   clockTicks() - t0 > dc.timeoutTicks) {
          reportError(dc, DERR_TIMEOUT);
          abortSh = 1;
        }
        if (abortSh) break;
      }
    }
    if (pending) {
      ok = false;
      break;
    }
    if (op.coll == LL_AG) {  // place every peer's payload in its block, and my own
      for (int q = 0; q < n; q++) {
        char* dst = recv + (uint64_t)q * nbytes;
        if (q == me) {
          if (dst != send) storePayload(dst, pk, payload(send, pk));
        } else {
          storePayload(dst, pk, llPayload(loadSeenLine16(myLL + llLineOffset(dc, c, par, q) + (pk - lo) * 16)));
        }
      }
      continue;
    }
    // Reduce: every rank sends to and polls every peer (that keeps the parity double-buffering safe, as
    // for AllReduce), only the root folds, in its ring order root+1, ..., root (reference reduce.h)
    if (!folds) continue;
    // pass 2: fold in the owner block's ring order (the lines stay valid until epoch + 2)
    const int owner = op.coll == LL_RS ? me
                    : op.coll == LL_REDUCE ? op.root
                    : (int)((pk * 8 / sizeof(T)) / op.chunk);  // an AllReduce payload never straddles blocks
    union { uint64_t u; T e[EPP]; } acc, x;
    for (int k = 0; k < n; k++) {
      int q = (owner + 1 + k) % n;
      if (q == me) {
        x.u = myV;
      } else {
        x.u = llPayload(loadSeenLine16(myLL + llLineOffset(dc, c, par, q) + (pk - lo) * 16));
      }
#pragma unroll
      for (int e = 0; e < EPP; e++) {
        T y = fn.pre(x.e[e]);
        acc.e[e] = k == 0 ? y : fn.red(y, acc.e[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < EPP; e++) acc.e[e] = fn.post(acc.e[e]);
    storePayload(recv, pk, acc.u);
  }
  __syncthreads();  // every payload of this op is folded before the next op's lines go out
  return ok && !abortSh;
}

// LL64: the LL128-class protocol (reference prims_ll128.h) on the line size MI355X stores atomically. A line
// is 64 bytes = 4 consecutive lanes x 16 bytes of one wave-instruction: lanes 0-2 carry 16 payload bytes,
// lane 3 carries 8 payload bytes and the 64-bit epoch flag, so 56 of every 64 bytes on the link are payload
// (LL: 8 of 16). The reader loads the whole line (4 lanes, one 16-byte system-scope load each) and accepts it
// once lane 3 sees the flag: that relies on the line arriving as one unit, which the store-atomicity probe
// measured for 64-byte segments (never torn) and refuted for 128-byte lines (torn in ~1.4 % of racing reads,
// DESIGN.md §10.1). Payloads, fold order, batching, epochs and parity double-buffering are the LL kernel's;
// the line area is its own (ll64LineOffset), so neither protocol can mistake the other's payload for a flag.

template <typename T, int OP>
__device__ __forceinline__ bool ll64ChannelOp(const DevComm& dc, const Red<T, OP>& fn, const LLOp& op, int c, int j,
                                              uint64_t e64, int& abortSh) {
  const int tid = threadIdx.x, lane = tid & 63, me = dc.rank, n = dc.nRanks;
  constexpr int EPP = 8 / sizeof(T);
  const uint32_t flag = (uint32_t)e64 ? (uint32_t)e64 : 1u;
  const int par = (int)(e64 & 1);
  // 32-bit indices (an op's payload space fits the line area, < 1 MiB): fewer live registers
  const uint32_t nbytes = (uint32_t)(op.count * sizeof(T));
  const uint32_t nLines = (nbytes + kLL64Payload - 1) / kLL64Payload;
  const uint32_t lo = min((uint32_t)j * (uint32_t)op.part, nLines), hi = min(lo + (uint32_t)op.part, nLines);
  const int u = tid & 3;  // my 16-byte unit of every line I touch (kThreads is a multiple of 4)
  const char* send = (const char*)op.send;
  char* recv = (char*)op.recv;
  auto payload = [&](const char* base, uint32_t pk) -> uint64_t {  // 8 bytes at any alignment, 0 past the end
    const char* p = base + pk * 8;
    const uintptr_t al = (uintptr_t)p;
    uint64_t v = 0;
    if (pk * 8 + 8 <= nbytes) {
      if ((al & 7) == 0) v = *(const uint64_t*)p;
      else if ((al & 3) == 0) v = ((const uint32_t*)p)[0] | ((uint64_t)((const uint32_t*)p)[1] << 32);
      else for (int b = 0; b < 8; b++) v |= (uint64_t)(unsigned char)p[b] << (8 * b);
    } else {
      for (uint32_t b = pk * 8; b < nbytes; b++) v |= (uint64_t)(unsigned char)base[b] << (8 * (b - pk * 8));
    }
    return v;
  };
  auto storePayload = [&](char* base, uint32_t pk, uint64_t v) {
    if (pk * 8 >= nbytes) return;
    char* p = base + pk * 8;
    const uintptr_t al = (uintptr_t)p;
    if (pk * 8 + 8 <= nbytes) {
      if ((al & 7) == 0) {
        *(uint64_t*)p = v;
      } else if ((al & 3) == 0) {
        ((uint32_t*)p)[0] = (uint32_t)v;
        ((uint32_t*)p)[1] = (uint32_t)(v >> 32);
      } else {
        for (int b = 0; b < 8; b++) p[b] = (char)(v >> (8 * b));
      }
    } else {
      for (uint32_t b = pk * 8; b < nbytes; b++) base[b] = (char)(v >> (8 * (b - pk * 8)));
    }
  };
  const uint64_t flag64 = ((uint64_t)flag << 32) | flag;
  // payload units of line L: 7L + 2u and 7L + 2u + 1 (u < 3), 7L + 6 (u == 3, beside the flag)
  constexpr int kUnits = kLL64Payload / 8;

  // send: unit u of lines [lo,hi) to every peer, one 16-byte write-through store per peer
  for (uint32_t i = lo * 4 + tid; i < hi * 4; i += kThreads) {
    const uint32_t pk = (i >> 2) * kUnits + 2 * u;
    const uint32_t off = (i - lo * 4) * 16;
    uint64_t v0 = 0, v1 = flag64;
    if (op.coll != LL_RS) {
      v0 = payload(send, pk);
      if (u < 3) v1 = payload(send, pk + 1);
    }
    for (int k = 1; k < n; k++) {
      int p = (me + k) % n;
      if (op.coll == LL_RS) {  // block p goes to its owner
        v0 = payload(send + (uint64_t)p * nbytes, pk);
        if (u < 3) v1 = payload(send + (uint64_t)p * nbytes, pk + 1);
      }
      char* base = (char*)dc.flags[p] + ll64LineOffset(dc, c, par, me) + off;
      storeRemote(base, u32x4{(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32)});
    }
  }
  __syncthreads();
  const uint64_t t0 = clockTicks();
  bool ok = true;
  const char* myLL = (const char*)dc.flags[me];
  const bool folds = op.coll != LL_AG && !(op.coll == LL_REDUCE && me != op.root);
  const char* mine = op.coll == LL_RS ? send + (uint64_t)me * nbytes : send;
  // pass 1: wait until every peer's line of every line this thread handles carries this epoch's flag (seen by
  // the group's lane 3). Lines are whole 4-lane groups and hi * 4 is a multiple of 4, so every lane a group
  // reads with __shfl is active in the same iteration. All lines are polled before any is folded, so a
  // thread with several lines waits once.
  for (uint32_t i = lo * 4 + tid; ok && i < hi * 4; i += kThreads) {
    const uint32_t off = (i - lo * 4) * 16;
    uint32_t pending = 0;
    for (int q = 0; q < n; q++)
      if (q != me) pending |= 1u << q;
    uint32_t spins = 0;
    while (true) {
      for (int q = 0; q < n; q++) {
        if (q == me) continue;
        const bool need = (pending >> q) & 1u;
        bool mineOk = true;
        if (need) {
          const u32x4 v = loadLine16(myLL + ll64LineOffset(dc, c, par, q) + off);
          mineOk = u != 3 || (v.z == flag && v.w == flag);
        }
        const bool lineOk = __shfl((int)mineOk, (lane & ~3) | 3) != 0;
        if (need && lineOk) pending &= ~(1u << q);
      }
      if (!__any(pending != 0)) break;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023) == 0) {
        if (__hip_atomic_load(dc.abortFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          reportError(dc, DERR_ABORT);
          abortSh = 1;
        } else if (__hip_atomic_load(dc.errorWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                   clockTicks() - t0 > dc.timeoutTicks) {
          reportError(dc, DERR_TIMEOUT);
          abortSh = 1;
        }
        if (abortSh) break;
      }
    }
    if (pending) ok = false;
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the re-reads below stay behind the polls
  // pass 2: re-read the lines (valid until epoch + 2) and place (AllGather) or fold them
  for (uint32_t i = lo * 4 + tid; ok && i < hi * 4; i += kThreads) {
    const uint32_t pk = (i >> 2) * kUnits + 2 * u;
    const uint32_t off = (i - lo * 4) * 16;
    if (op.coll == LL_AG) {  // place every peer's payload in its block, and my own
      for (int q = 0; q < n; q++) {
        char* dst = recv + (uint64_t)q * nbytes;
        uint64_t v0, v1;
        if (q == me) {
          if (dst == send) continue;
          v0 = payload(send, pk);
          v1 = u < 3 ? payload(send, pk + 1) : 0;
        } else {
          const u32x4 v = loadSeenLine16(myLL + ll64LineOffset(dc, c, par, q) + off);
          v0 = v.x | ((uint64_t)v.y << 32);
          v1 = v.z | ((uint64_t)v.w << 32);
        }
        storePayload(dst, pk, v0);
        if (u < 3) storePayload(dst, pk + 1, v1);
      }
      continue;
    }
    if (!folds) continue;  // Reduce: only the root folds, in its ring order root+1, ..., root
    // each payload folds in its owner block's ring order; both of my payloads share the owner except at a
    // block boundary, where the two are folded in separate passes
    const bool two = u < 3 && (pk + 1) * 8 < nbytes;
    auto ownerOf = [&](uint32_t q8) -> int {
      return op.coll == LL_RS ? me : op.coll == LL_REDUCE ? op.root : (int)((q8 * 8 / sizeof(T)) / op.chunk);
    };
    const int own0 = ownerOf(pk), own1 = two ? ownerOf(pk + 1) : own0;
    // source k of the fold order: my own payloads or peer q's line; the next source's load is issued before
    // the current one is folded
    auto fetch = [&](int owner, int k) -> u32x4 {
      const int q = (owner + 1 + k) % n;
      if (q == me) {
        const uint64_t a = payload(mine, pk), b = two ? payload(mine, pk + 1) : 0;
        return u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
      }
      return loadSeenLine16(myLL + ll64LineOffset(dc, c, par, q) + off);
    };
    // fold payload h (0: low 8 bytes of the unit, 1: high 8 bytes) in owner's order
    auto foldOne = [&](int owner, int h) {
      union { uint64_t u; T e[EPP]; } acc, x;
      u32x4 nxt = fetch(owner, 0);
      for (int k = 0; k < n; k++) {
        const u32x4 cur = nxt;
        if (k + 1 < n) nxt = fetch(owner, k + 1);
        x.u = h ? (cur.z | ((uint64_t)cur.w << 32)) : (cur.x | ((uint64_t)cur.y << 32));
#pragma unroll
        for (int e = 0; e < EPP; e++) {
          T y = fn.pre(x.e[e]);
          acc.e[e] = k == 0 ? y : fn.red(y, acc.e[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < EPP; e++) acc.e[e] = fn.post(acc.e[e]);
      storePayload(recv, pk + h, acc.u);
    };
    // both payloads of the unit in one pass (same owner: everywhere but at a block boundary); 1-byte types
    // unpack 8 elements per payload and always fold one payload per pass to stay within the register budget
    if constexpr (sizeof(T) > 1) {
      if (two && own0 == own1) {
        union { uint64_t u; T e[EPP]; } acc0, acc1, x0, x1;
        u32x4 nxt = fetch(own0, 0);
        for (int k = 0; k < n; k++) {
          const u32x4 cur = nxt;
          if (k + 1 < n) nxt = fetch(own0, k + 1);
          x0.u = cur.x | ((uint64_t)cur.y << 32);
          x1.u = cur.z | ((uint64_t)cur.w << 32);
#pragma unroll
          for (int e = 0; e < EPP; e++) {
            T y0 = fn.pre(x0.e[e]), y1 = fn.pre(x1.e[e]);
            acc0.e[e] = k == 0 ? y0 : fn.red(y0, acc0.e[e]);
            acc1.e[e] = k == 0 ? y1 : fn.red(y1, acc1.e[e]);
          }
        }
#pragma unroll
        for (int e = 0; e < EPP; e++) {
          acc0.e[e] = fn.post(acc0.e[e]);
          acc1.e[e] = fn.post(acc1.e[e]);
        }
        storePayload(recv, pk, acc0.u);
        storePayload(recv, pk + 1, acc1.u);
        continue;
      }
    }
    foldOne(own0, 0);
    if (two) foldOne(own1, 1);
  }
  __syncthreads();  // every payload of this op is folded before the next op's lines go out
  return ok && !abortSh;
}

// One launch runs a batch of LL ops (a single ReduceScatter / AllGather, or up to 32 AllReduces); op k occupies channels [chOff_k, chOff_k + nch_k) mod
// llChannels, so the small ops of a batch land on different channels and run in parallel (one
// round trip for the batch). A channel runs its ops in batch order and its epoch advances once per op
// it takes part in; all ranks build the same batch, so epochs agree.
template <typename T, int OP, int K, int P>
__global__ void __launch_bounds__(kThreads) kCoResident llKernel(LLArgs<K> a) {
  __shared__ int abortSh;
  const DevComm& dc = *a.comm;
  const int c = blockIdx.x;
  if (threadIdx.x == 0) abortSh = 0;
  uint64_t opArg = a.redArg;
  if (a.redArgPtr) {
    opArg = 0;
    __builtin_memcpy(&opArg, a.redArgPtr, sizeof(T));
  }
  const Red<T, OP> fn(opArg);
  uint64_t e64 = a.counters[ctrIndex(c, CTR_LL, 0)];
  __syncthreads();
  const int L = dc.llChannels;
  // the ops this channel runs, in batch order: one word of the arguments (host-built from the ops' channel
  // ranges). Walking every op's range instead cost ≈ 0.37 µs per op of the batch on MI355X (32 x 4 KiB:
  // 16.2 µs vs 5.6 µs for one 128 KiB op; tests/native/nccl_perf -G): each descriptor is its own line of the
  // argument block, and every work-group read them all.
  uint32_t mine = K == 1 ? 1u : a.chMask[c];
  while (mine) {
    const int k = K == 1 ? 0 : __builtin_ctz(mine);
    mine &= mine - 1;
    // the op's descriptor, loaded once (k is uniform: one burst of scalar loads) — referenced in place through a
    // dynamic index into the kernel arguments, its fields were re-read inside the op's loops
    const LLOp o = a.ops[k];
    const int j = (c - o.chOff + L) % L;  // op k runs on channels chOff, chOff+1, ... (mod L)
    if (j >= o.nch) break;                // (a lone op's grid is its channel count; a batch's masks say so)
    e64++;
    // one protocol per launch (a batch holds ops of one protocol): each kernel keeps its own register budget
    const bool ok = P == LLP_LL64 ? ll64ChannelOp<T, OP>(dc, fn, o, c, j, e64, abortSh)
                                  : llChannelOp<T, OP>(dc, fn, o, c, j, e64, abortSh);
    if (!ok) break;
  }
  if (threadIdx.x == 0) a.counters[ctrIndex(c, CTR_LL, 0)] = e64;
}

// ------------------------------------------------------------------------------------ symmetric windows
//
// Zero-copy collectives over registered symmetric windows (reference src/device/symmetric/all_reduce.cuh,
// reduce_scatter.cuh, all_gather.cuh: LSA barrier arrive at entry, wait before touching peers, sync at
// exit). Every rank's buffers are mapped here, so there is no staging: per channel
//   ENTER  tell every peer my inputs are ready (my kernel started: stream order), wait for theirs;
//   RS     the owner of block q pulls block q's channel part from all n inputs, folds it in the
//          reference's ring order (q+1, ..., q) and stores it in its own output;
//   MID    (AllReduce) publish that part (system release) and wait until every owner has published;
//   AG     pull the other n-1 reduced parts from the owners' outputs into my output;
//   DONE   tell every peer I finished reading its buffers and wait until all peers have: only then
//          may the stream reuse my buffers.
// Only remote LOADS cross xGMI (plus flag stores): user buffers are never written remotely, so no
// peer's L2 can hold a stale copy of bytes written behind its back; remote bytes are read after a
// system-scope acquire. Link bytes are those of the staged path, local HBM traffic drops from
// 2S + 4(n-1)S/n to about 3S, and one handshake round replaces the per-slice credit protocol.
// The epoch of each channel lives in device memory (counters[c][CTR_SYM]), so graphs replay.
enum SymColl { SYM_AR = 0, SYM_AR1 = 1, SYM_RS = 2, SYM_AG = 3 };

struct SymShared {
  ChanState st;
  WaitProbe probe;  // ENTER wait: a peer's staged-kernel flags beyond what this rank consumed are a mismatch
  const char* srcPtr[NCCL_AMD_MAX_RANKS];
  uint64_t want[NCCL_AMD_MAX_RANKS];
  uint64_t* sigPtr[NCCL_AMD_MAX_RANKS];
  uint64_t sigVal[NCCL_AMD_MAX_RANKS];
  char* pushPtr[1];
  const char* send[NCCL_AMD_MAX_RANKS];  // every rank's buffers as mapped here (windows: from the arguments;
  char* recv[NCCL_AMD_MAX_RANKS];        // registered buffers: exchanged at entry)
  int aligned;
};

// Every lane i < n (i != me) stores `e` into peer i's flag word [c][kind][me]; REL publishes my prior stores.
__device__ __forceinline__ void symSignal(const DevComm& dc, SymShared& sh, int c, int kind, uint64_t e, bool REL) {
  const int tid = threadIdx.x, me = dc.rank;
  if (tid < NCCL_AMD_MAX_RANKS) {
    bool peer = tid < dc.nRanks && tid != me;
    sh.sigVal[tid] = peer ? e : 0;
    sh.sigPtr[tid] = peer ? dc.flags[tid] + flagIndex(c, kind, me) : nullptr;
  }
  __syncthreads();
  signalAll(sh.sigPtr, sh.sigVal, NCCL_AMD_MAX_RANKS, REL);
  __syncthreads();
}

__device__ __forceinline__ bool symWait(const DevComm& dc, SymShared& sh, int c, int kind, uint64_t e, bool ACQ) {
  const int tid = threadIdx.x, me = dc.rank;
  if (tid < NCCL_AMD_MAX_RANKS) sh.want[tid] = (tid < dc.nRanks && tid != me) ? e : 0;
  if (tid == 0 && kind == FLG_SYM_ENTER) {  // (after ENTER every rank is known to run this kernel)
    const int fk[3] = {FLG_RS_READY, FLG_AG_READY, FLG_PULL_READY}, ck[3] = {CTR_RECV_RS, CTR_RECV_AG, CTR_PULL_GOT};
    for (int k = 0; k < 3; k++) {
      sh.probe.flag[k] = dc.flags[me] + flagIndex(c, fk[k], 0);
      sh.probe.seen[k] = dc.counters + ctrIndex(c, ck[k], 0);
    }
  }
  __syncthreads();
  const uint64_t* base = dc.flags[me] + flagIndex(c, kind, 0);
  return kind == FLG_SYM_ENTER ? waitAll<PROBE_SYM>(dc, sh.st, base, sh.want, ACQ, &sh.probe)
                               : waitAll(dc, sh.st, base, sh.want, ACQ);
}

template <typename T, int OP, int COLL>
__global__ void __launch_bounds__(kThreads) kCoResident symKernel(SymArgs a) {
  __shared__ SymShared sh;
  const DevComm& dc = *a.comm;
  const int tid = threadIdx.x, c = blockIdx.x, me = dc.rank, n = dc.nRanks;
  constexpr uint64_t ts = sizeof(T);
  if (tid == 0) sh.st.abort = 0;
  const uint64_t e = dc.counters[ctrIndex(c, CTR_SYM, 0)] + 1;
  uint64_t opArg = a.redArg;
  if (a.redArgPtr) {
    opArg = 0;
    __builtin_memcpy(&opArg, a.redArgPtr, sizeof(T));
  }
  const Red<T, OP> fn(opArg);
  // Registered mode reads peers' buffers at the pointers they hand over at ENTER. After a device error of this comm (a
  // kernel mismatch, a timeout) the ranks' epochs no longer match: an ENTER wait could pass on a peer's flag of an older
  // collective and read pointers whose mappings are gone. The error word is only written by this comm's kernels, which
  // precede this one in stream order, so every workgroup reads the same value and leaves at once.
  if (a.regMode && __hip_atomic_load(dc.errorWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != DERR_NONE) return;
  if (tid < NCCL_AMD_MAX_RANKS) {
    sh.send[tid] = a.send[tid];
    sh.recv[tid] = a.recv[tid];
    // registered buffers: hand rank tid MY buffers as mapped in its address space (its REG words of this
    // channel; read by it after my ENTER below, which signalAll orders behind these stores' completion)
    if (a.regMode && tid < n && tid != me) {
      storeFlag(dc.flags[tid] + flagIndex(c, FLG_REG_SEND, me), (uint64_t)a.send[tid]);
      storeFlag(dc.flags[tid] + flagIndex(c, FLG_REG_RECV, me), (uint64_t)a.recv[tid]);
    }
  }
  bool aligned = a.aligned != 0;
  // wtPublish: what peers read from my output (AR: my reduced part; AG: my own block) is stored system-scope
  // write-through, so nothing of it sits dirty in this XCD's L2 and the signal that publishes it needs no
  // L2 write-back (buffer_wbl2), only the store drain — as the staged path's pushes
  const bool wt = a.wtPublish != 0;
  auto blockLen = [&](int q) -> uint64_t {
    if (COLL == SYM_RS || COLL == SYM_AG) return a.chunk;
    uint64_t b = (uint64_t)q * a.chunk;
    return b >= a.count ? 0 : min(a.chunk, a.count - b);
  };
  auto partOf = [&](uint64_t len, uint64_t& lo, uint64_t& hi) {
    lo = min((uint64_t)c * a.part, len);
    hi = min(lo + a.part, len);
  };
  bool ok;
  bool agRel = false;  // AG: publish my block with an L2 write-back (no write-through copy of it was made)
  if (COLL == SYM_AG) {
    // AllGather: my own block goes into my output BEFORE entry (skipped in place), so every peer pulls block
    // q from rank q's output. No rank needs to know whether a peer runs in place or out of place (ranks may
    // mix them), and a sendbuff outside any window is fine: only outputs are read remotely.
    uint64_t lo, hi;
    partOf(a.chunk, lo, hi);
    char* dst = a.recv[me] + ((uint64_t)me * a.chunk + lo) * ts;
    const char* src = a.send[me] + lo * ts;
    // registered buffers: only my own pointers are known here, alignment of the copy is decided by them
    if (a.regMode) aligned = aligned && (((uintptr_t)a.recv[me] | (uintptr_t)a.send[me]) & 15) == 0;
    if (dst != src) {
      if (wt) copyRange<T, true>(dst, src, (hi - lo) * ts, aligned);
      else copyRange<T, false>(dst, src, (hi - lo) * ts, aligned);
    }
    // in place, the block was written by the caller's earlier kernels: keep the write-back release for it
    agRel = !wt || dst == src || a.relFence;
  }
  symSignal(dc, sh, c, FLG_SYM_ENTER, e, agRel);  // AG: publishes that block
  ok = symWait(dc, sh, c, FLG_SYM_ENTER, e, true);
  if (a.regMode) {
    // every peer stored its buffers (as mapped here) before its ENTER: read them, then decide the access
    // width from ALL ranks' pointers — the same set on every rank, so every rank takes the same path
    if (tid < n && tid != me) {
      sh.send[tid] = (const char*)loadFlag(dc.flags[me] + flagIndex(c, FLG_REG_SEND, tid));
      sh.recv[tid] = (char*)loadFlag(dc.flags[me] + flagIndex(c, FLG_REG_RECV, tid));
    }
    __syncthreads();
    if (tid == 0) {
      uintptr_t al = 0;
      for (int r = 0; r < n; r++) al |= (uintptr_t)sh.recv[r] | (COLL == SYM_AG ? 0 : (uintptr_t)sh.send[r]);
      sh.aligned = a.aligned != 0 && (al & 15) == 0;
    }
    __syncthreads();
    aligned = sh.aligned != 0;
  }
  if (ok && COLL == SYM_AR1) {
    // one-shot: fold my channel's portion of the whole buffer from all n inputs, owner block by block
    uint64_t lo, hi;
    partOf(a.count, lo, hi);
    for (uint64_t x = lo; x < hi;) {
      const int owner = (int)(x / a.chunk);
      const uint64_t end = min(hi, (uint64_t)(owner + 1) * a.chunk);
      if (tid == 0)
        for (int k = 0; k < n; k++) sh.srcPtr[k] = sh.send[(owner + 1 + k) % n] + x * ts;
      __syncthreads();
      foldRange<T, OP>(fn, n, sh.srcPtr, end - x, sh.recv[me] + x * ts, nullptr, 0, aligned);
      __syncthreads();
      x = end;
    }
  } else if (ok && COLL != SYM_AG) {
    // RS: fold my block's channel part; fold order owner+1, ..., owner (all_reduce.h:43-66)
    uint64_t lo, hi;
    partOf(blockLen(me), lo, hi);
    if (tid == 0)
      for (int k = 0; k < n; k++) sh.srcPtr[k] = sh.send[(me + 1 + k) % n] + ((uint64_t)me * a.chunk + lo) * ts;
    __syncthreads();
    char* dst = COLL == SYM_RS ? sh.recv[me] + lo * ts : sh.recv[me] + ((uint64_t)me * a.chunk + lo) * ts;
    const bool push = COLL == SYM_AR && wt;  // peers read it in the pull phase
    if (tid == 0) sh.pushPtr[0] = dst;
    __syncthreads();
    foldRange<T, OP>(fn, n, sh.srcPtr, hi - lo, push ? nullptr : dst, sh.pushPtr, push ? 1 : 0, aligned);
    __syncthreads();
  }
  if (ok && COLL == SYM_AR) {
    symSignal(dc, sh, c, FLG_SYM_MID, e, !wt || a.relFence);  // my reduced part is in my output: publish it
    ok = symWait(dc, sh, c, FLG_SYM_MID, e, true);
  }
  if (ok && (COLL == SYM_AR || COLL == SYM_AG)) {
    // pull every other rank's block part from its output (AR: its reduced block; AG: its input block)
    for (int k = 1; k < n; k++) {
      const int q = chanPeer(me, n, c, k);  // staggered by channel: all links busy
      uint64_t lo, hi;
      partOf(blockLen(q), lo, hi);
      const uint64_t off = ((uint64_t)q * a.chunk + lo) * ts;
      copyRange<T, false>(sh.recv[me] + off, sh.recv[q] + off, (hi - lo) * ts, aligned);
    }
    __syncthreads();
  }
  if (ok) {
    symSignal(dc, sh, c, FLG_SYM_DONE, e, false);  // drained: I no longer read any peer's buffers
    ok = symWait(dc, sh, c, FLG_SYM_DONE, e, false);
  }
  (void)ok;  // on failure the error word is set and the epoch still advances (the comm is unusable)
  if (tid == 0) dc.counters[ctrIndex(c, CTR_SYM, 0)] = e;
}

template <typename T, int OP>
inline ncclResult_t launchSymTyped(const SymPlan& p) {
  switch (p.coll) {
    case SYM_AR: NCCL_AMD_LAUNCH((symKernel<T, OP, SYM_AR>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
    case SYM_AR1: NCCL_AMD_LAUNCH((symKernel<T, OP, SYM_AR1>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
    case SYM_RS: NCCL_AMD_LAUNCH((symKernel<T, OP, SYM_RS>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
    case SYM_AG: NCCL_AMD_LAUNCH((symKernel<T, 0, SYM_AG>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
  }
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

template <typename T>
inline ncclResult_t launchSymOp(const SymPlan& p) {
  switch (p.devOp) {
    case DEV_SUM: return launchSymTyped<T, DEV_SUM>(p);
    case DEV_PROD: return launchSymTyped<T, DEV_PROD>(p);
    case DEV_MINMAX: return launchSymTyped<T, DEV_MINMAX>(p);
    case DEV_PREMULSUM: return launchSymTyped<T, DEV_PREMULSUM>(p);
    default: break;
  }
  WARN("internal: op %d unsupported for this type", p.devOp);
  return ncclInternalError;
}
template <typename T>
inline ncclResult_t launchSymIntOp(const SymPlan& p) {
  if (p.devOp == DEV_SUMPOSTDIV) return launchSymTyped<T, DEV_SUMPOSTDIV>(p);
  return launchSymOp<T>(p);
}

// ------------------------------------------------------------------------------------ nRanks == 1

// PreMulSum on one rank (reference onerank.cu:14-47): out = post(pre(in)). Like the nRanks == 1 copy (kernels.hip):
// 16-byte packs, 2 per thread, one 8 KiB tile per 256-thread workgroup (grid-stride past the grid), nontemporal
// loads and system-scope write-through buffer stores; element-wise for unaligned buffers and the
// < 16-byte tail.
template <typename T, int OP>
__global__ void __launch_bounds__(256) oneRankKernel(T* dst, const T* src, uint64_t n, uint64_t arg,
                                                     const void* argPtr, int aligned) {
  uint64_t a = arg;
  if (argPtr) {
    a = 0;
    __builtin_memcpy(&a, argPtr, sizeof(T));
  }
  const Red<T, OP> fn(a);
  constexpr int EPP = 16 / sizeof(T), U = 2;
  const uint64_t npk = aligned ? n / EPP : 0;
  const u32x4* s = (const u32x4*)src;
  for (uint64_t t0 = (uint64_t)blockIdx.x * 256 * U; t0 < npk; t0 += (uint64_t)gridDim.x * 256 * U) {
    PackU<T> v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (t0 + threadIdx.x + u * 256 < npk) v[u].v = __builtin_nontemporal_load(s + t0 + threadIdx.x + u * 256);
    const __amdgpu_buffer_rsrc_t rd = remoteRsrc((u32x4*)dst + t0);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (t0 + threadIdx.x + u * 256 < npk) {
#pragma unroll
        for (int e = 0; e < EPP; e++) v[u].e[e] = fn.post(fn.pre(v[u].e[e]));
        __builtin_amdgcn_raw_buffer_store_b128(v[u].v, rd, (threadIdx.x + u * 256) * 16u, 0, kSysWriteThrough);
      }
  }
  for (uint64_t i = npk * EPP + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = fn.post(fn.pre(src[i]));
}

// ------------------------------------------------------------------------------------ host launcher

// LL launch with the smallest argument block that holds the batch (1, 8 or 32 ops)
template <typename T, int OP, int K>
inline void launchLLK(const LaunchPlan& p) {
  LLArgs<K> a;
  a.comm = p.ll.comm;
  a.counters = p.ll.counters;
  a.redArg = p.ll.redArg;
  a.redArgPtr = p.ll.redArgPtr;
  a.nOps = p.ll.nOps;
  for (int k = 0; k < p.ll.nOps && k < K; k++) a.ops[k] = p.ll.ops[k];
  if constexpr (K > 1) __builtin_memcpy(a.chMask, p.ll.chMask, sizeof(a.chMask));
  if (p.ll.ops[0].proto == LLP_LL64)
    NCCL_AMD_LAUNCH((llKernel<T, OP, K, LLP_LL64>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, a);
  else
    NCCL_AMD_LAUNCH((llKernel<T, OP, K, LLP_LL>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, a);
}
template <typename T, int OP>
inline void launchLL(const LaunchPlan& p) {
  if (p.ll.nOps <= 1) launchLLK<T, OP, 1>(p);
  else if (p.ll.nOps <= 8) launchLLK<T, OP, 8>(p);
  else launchLLK<T, OP, kMaxLLBatch>(p);
}

// the staged kernel: one op, or a group batch (collBatchKernel)
template <typename T, int OP, int COLL>
inline void launchColl(const LaunchPlan& p) {
  if constexpr (COLL != COLL_ARREF) {  // reference-order AllReduces are never batched (enqueue.cc batchable)
    if (p.batch.nOps > 1) {
      NCCL_AMD_LAUNCH((collBatchKernel<T, OP, COLL>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.batch);
      return;
    }
  }
  NCCL_AMD_LAUNCH((collKernel<T, OP, COLL>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args);
}

template <typename T, int OP>
inline ncclResult_t launchTyped(const LaunchPlan& p) {
  if (p.algo == ALGO_ONERANK) {
    const int aligned = (((uintptr_t)p.args.recvbuff | (uintptr_t)p.args.sendbuff) & 15) == 0;
    constexpr uint64_t kTile = 256 * 2 * (16 / sizeof(T));  // elements per 8 KiB tile
    const uint64_t units = aligned ? (p.args.count + kTile - 1) / kTile : (p.args.count + 255) / 256;
    int grid = (int)std::min<uint64_t>(aligned ? (1u << 20) : 1024, units);
    if (grid < 1) grid = 1;
    NCCL_AMD_LAUNCH((oneRankKernel<T, OP>), dim3(grid), dim3(256), 0, p.stream, (T*)p.args.recvbuff,
                       (const T*)p.args.sendbuff, p.args.count, p.args.redArg, p.args.redArgPtr, aligned);
    HIPCHECK(hipGetLastError());
    return ncclSuccess;
  }
  if (p.algo == ALGO_PIPE) {  // ring / chain (pipe.h); AllGather is type-erased (launchKernGather)
    switch (p.pipeKind) {
      case PIPE_RING_AR: NCCL_AMD_LAUNCH((pipeKernel<T, OP, PIPE_RING_AR>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
      case PIPE_RING_RS: NCCL_AMD_LAUNCH((pipeKernel<T, OP, PIPE_RING_RS>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
      case PIPE_RING_AG: NCCL_AMD_LAUNCH((pipeKernel<T, 0, PIPE_RING_AG>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
      case PIPE_CHAIN_AR: NCCL_AMD_LAUNCH((pipeKernel<T, OP, PIPE_CHAIN_AR>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
      case PIPE_CHAIN_REDUCE: NCCL_AMD_LAUNCH((pipeKernel<T, OP, PIPE_CHAIN_REDUCE>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args); break;
      default: return ncclInternalError;
    }
    HIPCHECK(hipGetLastError());
    return ncclSuccess;
  }
  switch (p.func) {
    case FUNC_ALLREDUCE:
      if (p.algo == ALGO_LL) launchLL<T, OP>(p);
      else if (p.algo == ALGO_ONESHOT) launchColl<T, OP, COLL_AR1>(p);
      else if (p.args.cbdLo) launchColl<T, OP, COLL_ARREF>(p);  // NCCL_AMD_REF_ORDER (planColl)
      else launchColl<T, OP, COLL_AR>(p);
      break;
    case FUNC_REDUCESCATTER:
      if (p.algo == ALGO_LL) launchLL<T, OP>(p);
      else launchColl<T, OP, COLL_RS>(p);
      break;
    case FUNC_REDUCE:
      if (p.algo == ALGO_LL) launchLL<T, OP>(p);
      else launchColl<T, OP, COLL_REDUCE>(p);
      break;
    case FUNC_ALLGATHER:
      if (p.algo == ALGO_LL) launchLL<T, 0>(p);
      else launchColl<T, 0, COLL_AG>(p);
      break;
    default: return ncclInternalError;
  }
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

template <typename T>
inline ncclResult_t launchOp(const LaunchPlan& p) {
  switch (p.devOp) {
    case DEV_SUM: return launchTyped<T, DEV_SUM>(p);
    case DEV_PROD: return launchTyped<T, DEV_PROD>(p);
    case DEV_MINMAX: return launchTyped<T, DEV_MINMAX>(p);
    case DEV_PREMULSUM: return launchTyped<T, DEV_PREMULSUM>(p);
    default: break;
  }
  WARN("internal: op %d unsupported for this type", p.devOp);
  return ncclInternalError;
}
template <typename T>
inline ncclResult_t launchIntOp(const LaunchPlan& p) {
  if (p.devOp == DEV_SUMPOSTDIV) return launchTyped<T, DEV_SUMPOSTDIV>(p);
  return launchOp<T>(p);
}

}  // namespace ncclamd
