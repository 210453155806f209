// kernels.hip — gfx950 device code of the reduction engine + the host-side launcher.
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
// Memory model: remote payload = `global_store_dwordx4 ... sc0 sc1` (system-scope
// write-through) into the peer's UNCACHED staging; every storing wave drains (s_waitcnt vmcnt(0)),
// the workgroup barriers, one lane issues a system release fence and then a system-scope flag
// store. The consumer polls its local flag with system-scope loads (one wave, s_sleep between polls,
// bounded by NCCL_AMD_SPIN_TIMEOUT_MS and the host abort word), then one system acquire
// (buffer_inv sc0 sc1), vmcnt(0), barrier, plain loads.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "core.h"
#include "numerics.h"

namespace ncclamd {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 512;  // 8 waves of 64 per channel workgroup

// ------------------------------------------------------------------------------------ primitives

__device__ __forceinline__ uint64_t clockTicks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void storeRemote(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void drainStores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

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

// Wave 0 waits until every selected flag word reaches its target. Returns false on timeout/abort.
// want[r] = 0 means "no wait for r". All threads must call (contains barriers).
__device__ bool waitAll(const DevComm& dc, ChanState& st, const uint64_t* flagBase, const uint64_t* target) {
  if (threadIdx.x < 64) {
    int lane = threadIdx.x;
    bool need = lane < dc.nRanks && target[lane] != 0;
    uint64_t t0 = clockTicks();
    uint32_t iter = 0;
    while (true) {
      bool ok = !need || loadFlag(flagBase + lane) >= target[lane];
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if ((++iter & 255) == 0) {
        bool bad = false;
        if (__hip_atomic_load(dc.abortFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          if (lane == 0) reportError(dc, DERR_ABORT);
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
    if (lane == 0) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // buffer_inv sc0 sc1 (system acquire)
    drainStores();
  }
  __syncthreads();
  return st.abort == 0;
}

// All storing waves drain, then wave-0 lane r releases and bumps flag[r] on every selected peer.
__device__ void signalAll(const DevComm& dc, uint64_t* const* remoteFlag, const uint64_t* value) {
  drainStores();
  __syncthreads();
  if (threadIdx.x < 64) {
    int lane = threadIdx.x;
    __atomic_thread_fence(__ATOMIC_RELEASE);  // buffer_wbl2 sc0 sc1 + vmcnt(0)
    drainStores();
    if (lane < dc.nRanks && value[lane] != 0) storeFlag(remoteFlag[lane], value[lane]);
  }
}

// ------------------------------------------------------------------------------------ data movement

// Copy [0,nbytes) from src to dst. Both 16-byte aligned when `aligned`; nbytes multiple of sizeof(T).
template <typename T, bool REMOTE>
__device__ __forceinline__ void copyRange(void* dst, const void* src, uint64_t nbytes, bool aligned) {
  if (aligned) {
    uint64_t npk = nbytes >> 4;
    const u32x4* s = (const u32x4*)src;
    u32x4* d = (u32x4*)dst;
    constexpr int U = 4;
    uint64_t i = threadIdx.x;
    for (; i + (U - 1) * kThreads < npk; i += U * kThreads) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s + i + u * kThreads);
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (REMOTE) storeRemote(d + i + u * kThreads, v[u]);
        else d[i + u * kThreads] = v[u];
      }
    }
    for (; i < npk; i += kThreads) {
      u32x4 v = __builtin_nontemporal_load(s + i);
      if (REMOTE) storeRemote(d + i, v);
      else d[i] = v;
    }
    uint64_t done = npk << 4;
    uint64_t tail = (nbytes - done) / sizeof(T);
    if (threadIdx.x < tail) {
      const T* st = (const T*)((const char*)src + done);
      T* dt = (T*)((char*)dst + done);
      dt[threadIdx.x] = st[threadIdx.x];
    }
  } else {
    uint64_t n = nbytes / sizeof(T);
    const T* s = (const T*)src;
    T* d = (T*)dst;
    for (uint64_t i = threadIdx.x; i < n; i += kThreads) d[i] = s[i];
  }
}

template <typename T>
union PackU {
  u32x4 v;
  T e[16 / sizeof(T)];
};

// Fold n sources into dst (and optionally into nPush remote copies). src[k] is the k-th source in
// fold order: acc = pre(src[0]); acc = red(pre(src[k]), acc) ...; out = post(acc).
template <typename T, int OP>
__device__ __forceinline__ void foldRange(const Red<T, OP>& fn, int n, const void* const* src, uint64_t nelem,
                                          void* dstLocal, void* const* dstPush, int nPush, bool aligned) {
  constexpr int EPP = 16 / sizeof(T);
  if (aligned) {
    uint64_t npk = nelem / EPP;
    for (uint64_t i = threadIdx.x; i < npk; i += kThreads) {
      PackU<T> v[NCCL_AMD_MAX_RANKS];
#pragma unroll
      for (int k = 0; k < NCCL_AMD_MAX_RANKS; k++)
        if (k < n) v[k].v = __builtin_nontemporal_load((const u32x4*)src[k] + i);
      PackU<T> acc;
#pragma unroll
      for (int e = 0; e < EPP; e++) acc.e[e] = fn.pre(v[0].e[e]);
#pragma unroll
      for (int k = 1; k < NCCL_AMD_MAX_RANKS; k++)
        if (k < n) {
#pragma unroll
          for (int e = 0; e < EPP; e++) acc.e[e] = fn.red(fn.pre(v[k].e[e]), acc.e[e]);
        }
#pragma unroll
      for (int e = 0; e < EPP; e++) acc.e[e] = fn.post(acc.e[e]);
      if (dstLocal) ((u32x4*)dstLocal)[i] = acc.v;
#pragma unroll
      for (int p = 0; p < NCCL_AMD_MAX_RANKS - 1; p++)
        if (p < nPush) storeRemote((u32x4*)dstPush[p] + i, acc.v);
    }
    uint64_t done = npk * EPP;
    uint64_t t = done + threadIdx.x;
    if (t < nelem) {
      T acc = fn.pre(((const T*)src[0])[t]);
      for (int k = 1; k < n; k++) acc = fn.red(fn.pre(((const T*)src[k])[t]), acc);
      acc = fn.post(acc);
      if (dstLocal) ((T*)dstLocal)[t] = acc;
      for (int p = 0; p < nPush; p++) ((T*)dstPush[p])[t] = acc;  // < 16 B: plain store, fenced below
    }
  } else {
    for (uint64_t t = threadIdx.x; t < nelem; t += kThreads) {
      T acc = fn.pre(((const T*)src[0])[t]);
      for (int k = 1; k < n; k++) acc = fn.red(fn.pre(((const T*)src[k])[t]), acc);
      acc = fn.post(acc);
      if (dstLocal) ((T*)dstLocal)[t] = acc;
      for (int p = 0; p < nPush; p++) ((T*)dstPush[p])[t] = acc;
    }
  }
}

// ------------------------------------------------------------------------------------ collective kernel

enum Coll { COLL_AR = 0, COLL_RS = 1, COLL_AG = 2, COLL_REDUCE = 3 };

// Element range [lo,hi) of block q handled by channel c at pipeline step s (offsets inside the block).
__device__ __forceinline__ void sliceRange(const CollArgs& a, int c, int s, uint64_t blockLen, uint64_t& lo,
                                           uint64_t& hi) {
  uint64_t pEnd = min((uint64_t)(c + 1) * a.part, blockLen);
  lo = min((uint64_t)c * a.part + (uint64_t)s * a.slice, pEnd);
  hi = min(lo + a.slice, pEnd);
}

template <typename T, int OP, int COLL>
__global__ void __launch_bounds__(kThreads) collKernel(CollArgs a) {
  __shared__ ChanState st;
  __shared__ uint64_t want[NCCL_AMD_MAX_RANKS];
  __shared__ uint64_t* rflag[NCCL_AMD_MAX_RANKS];
  const DevComm& dc = *a.comm;
  const int c = blockIdx.x;
  const int me = dc.rank, n = dc.nRanks;
  const int tid = threadIdx.x;
  constexpr uint64_t ts = sizeof(T);

  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    st.ctr[k][r] = dc.counters[ctrIndex(c, k, r)];
  }
  if (tid == 0) st.abort = 0;
  __syncthreads();

  uint64_t opArg = a.redArg;
  if (a.redArgPtr) {  // ncclScalarDevice PreMulSum: dereference at run time (reference onerank.cu:31-41)
    opArg = 0;
    __builtin_memcpy(&opArg, a.redArgPtr, ts);
  }
  const Red<T, OP> fn(opArg);
  const bool aligned = a.aligned != 0;
  const uint64_t* myFlags = dc.flags[me];
  const int nSlots = dc.nSlots;
  // total length of block q (AR: last blocks may be short or empty)
  auto blockLen = [&](int q) -> uint64_t {
    if (COLL == COLL_AR || COLL == COLL_REDUCE) {
      uint64_t b = (uint64_t)q * a.chunk;
      return b >= a.count ? 0 : min(a.chunk, a.count - b);
    }
    return a.chunk;
  };
  const bool isRoot = (COLL != COLL_REDUCE) || me == a.root;

  for (int step = 0; step < a.nSteps; step++) {
    // ---------------- phase A: scatter input block p to owner p (AR, RS, REDUCE)
    if (COLL != COLL_AG) {
      if (tid < NCCL_AMD_MAX_RANKS) {
        // credit: peer p must have consumed the slice that used this slot nSlots sends ago
        uint64_t s = st.ctr[CTR_SEND_RS][tid];
        want[tid] = (tid < n && tid != me && s + 1 > (uint64_t)nSlots) ? s + 1 - nSlots : 0;
      }
      __syncthreads();
      if (!waitAll(dc, st, myFlags + flagIndex(c, FLG_RS_ACK, 0), want)) break;
      for (int k = 1; k < n; k++) {
        int p = (me + k) % n;
        uint64_t lo, hi;
        sliceRange(a, c, step, blockLen(p), lo, hi);
        int slot = (int)(st.ctr[CTR_SEND_RS][p] % nSlots);
        char* dst = dc.staging[p] + stagingOffset(dc, c, STG_RS, slot, me);
        const char* src = (const char*)a.sendbuff + ((uint64_t)p * a.chunk + lo) * ts;
        copyRange<T, true>(dst, src, (hi - lo) * ts, aligned);
      }
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool act = tid < n && tid != me;
        want[tid] = act ? st.ctr[CTR_SEND_RS][tid] + 1 : 0;
        rflag[tid] = act ? dc.flags[tid] + flagIndex(c, FLG_RS_READY, me) : nullptr;
      }
      __syncthreads();
      signalAll(dc, rflag, want);
      __syncthreads();
      if (tid < n && tid != me) st.ctr[CTR_SEND_RS][tid]++;
      __syncthreads();
    }

    // ---------------- phase B: reduce my block (AR, RS, REDUCE) or publish my block (AG)
    {
      // wait for: RS data from every peer (not AG); AG credits on every peer I push to
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool peer = tid < n && tid != me;
        want[tid] = (peer && COLL != COLL_AG) ? st.ctr[CTR_RECV_RS][tid] + 1 : 0;
      }
      __syncthreads();
      if (COLL != COLL_AG && !waitAll(dc, st, myFlags + flagIndex(c, FLG_RS_READY, 0), want)) break;
      bool pushAll = (COLL == COLL_AR || COLL == COLL_AG);
      bool pushRoot = (COLL == COLL_REDUCE && !isRoot);
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool dstPeer = tid < n && tid != me && (pushAll || (pushRoot && tid == a.root));
        uint64_t s = st.ctr[CTR_SEND_AG][tid];
        want[tid] = (dstPeer && s + 1 > (uint64_t)nSlots) ? s + 1 - nSlots : 0;
      }
      __syncthreads();
      if ((pushAll || pushRoot) && !waitAll(dc, st, myFlags + flagIndex(c, FLG_AG_ACK, 0), want)) break;

      uint64_t lo, hi;
      sliceRange(a, c, step, blockLen(me), lo, hi);
      uint64_t nelem = hi - lo;
      void* push[NCCL_AMD_MAX_RANKS];
      int nPush = 0;
      for (int k = 1; k < n; k++) {
        int p = (me + k) % n;
        if (pushAll || (pushRoot && p == a.root)) {
          int slot = (int)(st.ctr[CTR_SEND_AG][p] % nSlots);
          push[nPush++] = dc.staging[p] + stagingOffset(dc, c, STG_AG, slot, me);
        }
      }
      if (COLL == COLL_AG) {
        const char* src = (const char*)a.sendbuff + lo * ts;
        for (int i = 0; i < nPush; i++) copyRange<T, true>(push[i], src, nelem * ts, aligned);
        char* dst = (char*)a.recvbuff + ((uint64_t)me * a.chunk + lo) * ts;
        if (dst != src) copyRange<T, false>(dst, src, nelem * ts, aligned);
      } else {
        // fold order: first = owner+1 (AR/RS, reference all_reduce.h:43-66) or root+1 (Reduce, reduce.h:34-52)
        int first = (COLL == COLL_REDUCE ? a.root + 1 : me + 1) % n;
        const void* src[NCCL_AMD_MAX_RANKS];
        for (int k = 0; k < n; k++) {
          int q = (first + k) % n;
          if (q == me) src[k] = (const char*)a.sendbuff + ((uint64_t)me * a.chunk + lo) * ts;
          else src[k] = dc.staging[me] + stagingOffset(dc, c, STG_RS, (int)(st.ctr[CTR_RECV_RS][q] % nSlots), q);
        }
        void* dstLocal = nullptr;
        if (COLL == COLL_AR) dstLocal = (char*)a.recvbuff + ((uint64_t)me * a.chunk + lo) * ts;
        else if (COLL == COLL_RS) dstLocal = (char*)a.recvbuff + lo * ts;
        else if (isRoot) dstLocal = (char*)a.recvbuff + ((uint64_t)me * a.chunk + lo) * ts;
        foldRange<T, OP>(fn, n, src, nelem, dstLocal, push, nPush, aligned);
      }
      // release: RS slots consumed (ack to each sender) + AG data ready at each destination
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool peer = tid < n && tid != me;
        bool dstPeer = peer && (pushAll || (pushRoot && tid == a.root));
        want[tid] = (peer && COLL != COLL_AG) ? st.ctr[CTR_RECV_RS][tid] + 1 : 0;
        rflag[tid] = (peer && COLL != COLL_AG) ? dc.flags[tid] + flagIndex(c, FLG_RS_ACK, me) : nullptr;
      }
      __syncthreads();
      signalAll(dc, rflag, want);
      __syncthreads();
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool peer = tid < n && tid != me;
        bool dstPeer = peer && (pushAll || (pushRoot && tid == a.root));
        want[tid] = dstPeer ? st.ctr[CTR_SEND_AG][tid] + 1 : 0;
        rflag[tid] = dstPeer ? dc.flags[tid] + flagIndex(c, FLG_AG_READY, me) : nullptr;
      }
      __syncthreads();
      signalAll(dc, rflag, want);
      __syncthreads();
      if (tid < n && tid != me) {
        if (COLL != COLL_AG) st.ctr[CTR_RECV_RS][tid]++;
        if (pushAll || (pushRoot && tid == a.root)) st.ctr[CTR_SEND_AG][tid]++;
      }
      __syncthreads();
    }

    // ---------------- phase C: gather the other blocks into the output (AR, AG, REDUCE at root)
    if (COLL == COLL_AR || COLL == COLL_AG || (COLL == COLL_REDUCE && isRoot)) {
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool peer = tid < n && tid != me;
        want[tid] = peer ? st.ctr[CTR_RECV_AG][tid] + 1 : 0;
      }
      __syncthreads();
      if (!waitAll(dc, st, myFlags + flagIndex(c, FLG_AG_READY, 0), want)) break;
      for (int k = 1; k < n; k++) {
        int q = (me + n - k) % n;
        uint64_t lo, hi;
        sliceRange(a, c, step, blockLen(q), lo, hi);
        const char* src = dc.staging[me] + stagingOffset(dc, c, STG_AG, (int)(st.ctr[CTR_RECV_AG][q] % nSlots), q);
        char* dst = (char*)a.recvbuff + ((uint64_t)q * a.chunk + lo) * ts;
        copyRange<T, false>(dst, src, (hi - lo) * ts, aligned);
      }
      // our loads have returned (data stored from registers) -> return the credits
      if (tid < NCCL_AMD_MAX_RANKS) {
        bool peer = tid < n && tid != me;
        want[tid] = peer ? st.ctr[CTR_RECV_AG][tid] + 1 : 0;
        rflag[tid] = peer ? dc.flags[tid] + flagIndex(c, FLG_AG_ACK, me) : nullptr;
      }
      __syncthreads();
      signalAll(dc, rflag, want);
      __syncthreads();
      if (tid < n && tid != me) st.ctr[CTR_RECV_AG][tid]++;
      __syncthreads();
    }
  }
  __syncthreads();
  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    dc.counters[ctrIndex(c, k, r)] = st.ctr[k][r];
  }
}

// ------------------------------------------------------------------------------------ nRanks == 1

// Streaming copy (reference onerank.cu:52-56 uses cudaMemcpyAsync; this is the hand-written
// replacement): 16 B per lane, U packs in flight per lane, grid-stride over 1 KiB wave tiles.
template <int U>
__global__ void __launch_bounds__(256) copyKernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                  uint64_t npk) {
  uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < npk; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * 256 < npk) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * 256 < npk) __builtin_nontemporal_store(v[u], dst + base + u * 256);
  }
}

__global__ void copyBytesKernel(char* dst, const char* src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// PreMulSum on one rank (reference onerank.cu:14-47): out = post(pre(in)).
template <typename T, int OP>
__global__ void __launch_bounds__(256) oneRankKernel(T* dst, const T* src, uint64_t n, uint64_t arg,
                                                     const void* argPtr) {
  uint64_t a = arg;
  if (argPtr) {
    a = 0;
    __builtin_memcpy(&a, argPtr, sizeof(T));
  }
  const Red<T, OP> fn(a);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = fn.post(fn.pre(src[i]));
}

// ------------------------------------------------------------------------------------ host launcher

template <typename T, int OP>
static ncclResult_t launchTyped(const LaunchPlan& p) {
  if (p.algo == ALGO_ONERANK) {
    int grid = (int)std::min<uint64_t>(1024, (p.args.count + 255) / 256);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((oneRankKernel<T, OP>), dim3(grid), dim3(256), 0, p.stream, (T*)p.args.recvbuff,
                       (const T*)p.args.sendbuff, p.args.count, p.args.redArg, p.args.redArgPtr);
    HIPCHECK(hipGetLastError());
    return ncclSuccess;
  }
  switch (p.func) {
    case FUNC_ALLREDUCE:
      hipLaunchKernelGGL((collKernel<T, OP, COLL_AR>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args);
      break;
    case FUNC_REDUCESCATTER:
      hipLaunchKernelGGL((collKernel<T, OP, COLL_RS>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args);
      break;
    case FUNC_REDUCE:
      hipLaunchKernelGGL((collKernel<T, OP, COLL_REDUCE>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args);
      break;
    case FUNC_ALLGATHER:
      hipLaunchKernelGGL((collKernel<T, 0, COLL_AG>), dim3(p.nChannels), dim3(kThreads), 0, p.stream, p.args);
      break;
  }
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

template <typename T>
static ncclResult_t launchOp(const LaunchPlan& p) {
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
static ncclResult_t launchIntOp(const LaunchPlan& p) {
  if (p.devOp == DEV_SUMPOSTDIV) return launchTyped<T, DEV_SUMPOSTDIV>(p);
  return launchOp<T>(p);
}

ncclResult_t launchCopy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (bytes == 0 || dst == src) return ncclSuccess;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    uint64_t npk = bytes >> 4;
    constexpr int U = 4;
    if (npk) {
      uint64_t tiles = (npk + 256 * U - 1) / (256 * U);
      int grid = (int)std::min<uint64_t>(tiles, (uint64_t)paramInt("NCCL_AMD_COPY_GRID", 2048));
      hipLaunchKernelGGL((copyKernel<U>), dim3(grid), dim3(256), 0, stream, (u32x4*)dst, (const u32x4*)src, npk);
      HIPCHECK(hipGetLastError());
    }
    uint64_t done = npk << 4;
    if (done < bytes) {
      hipLaunchKernelGGL(copyBytesKernel, dim3(1), dim3(64), 0, stream, (char*)dst + done, (const char*)src + done,
                         (uint64_t)(bytes - done));
      HIPCHECK(hipGetLastError());
    }
    return ncclSuccess;
  }
  int grid = (int)std::min<uint64_t>(2048, (bytes + 255) / 256);
  hipLaunchKernelGGL(copyBytesKernel, dim3(grid), dim3(256), 0, stream, (char*)dst, (const char*)src, (uint64_t)bytes);
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

ncclResult_t launchPlan(const LaunchPlan& p) {
  if (p.algo == ALGO_COPY) return launchCopy(p.args.recvbuff, p.args.sendbuff, p.bytes, p.stream);
  if (p.func == FUNC_ALLGATHER) {
    switch (p.eltSize) {
      case 1: return launchTyped<uint8_t, 0>(p);
      case 2: return launchTyped<uint16_t, 0>(p);
      case 4: return launchTyped<uint32_t, 0>(p);
      default: return launchTyped<uint64_t, 0>(p);
    }
  }
  switch (p.datatype) {
    case ncclInt8: case ncclUint8: return launchIntOp<uint8_t>(p);
    case ncclInt32: case ncclUint32: return launchIntOp<uint32_t>(p);
    case ncclInt64: case ncclUint64: return launchIntOp<uint64_t>(p);
    case ncclFloat16: return launchOp<half_t>(p);
    case ncclBfloat16: return launchOp<bf16_t>(p);
    case ncclFloat32: return launchOp<float>(p);
    case ncclFloat64: return launchOp<double>(p);
    case ncclFloat8e4m3: return launchOp<e4m3_t>(p);
    case ncclFloat8e5m2: return launchOp<e5m2_t>(p);
    default: break;
  }
  return ncclInvalidArgument;
}

}  // namespace ncclamd
