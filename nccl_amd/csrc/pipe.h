// pipe.h — the reference's own point-to-point pipeline algorithms on the staging/credit machinery of
// kernels.h: the RING (NCCL_ALGO=RING) and the intra-node CHAIN that the reference's TREE algorithm is on a
// single node (NCCL_ALGO=TREE). Included by kernels.h.
//
// Reference: src/device/all_reduce.h:13-83 (runRing: send, n-2 x recvReduceSend, recvReduceCopySend,
// n-2 x recvCopySend, recv), :86-143 (runTreeUpDown: reduce up the tree, then broadcast down),
// src/device/reduce_scatter.h:13-79, all_gather.h:13-114, reduce.h:13-76 (chain to the root),
// src/graph/connect.cc:53-63 (intra-node tree = chain: treeIntra[i].up = treeIntra[i-1], root treeIntra[0]).
//
// Each rank exchanges data with ONE neighbour per direction (prev / next in the ring, up / down in the chain)
// instead of all n-1 peers: every hop moves one staging slot over one xGMI link, with the same per-(channel,
// peer) step counters, READY / ACK flags and nSlots credit window as the direct kernel (so the three
// algorithms can follow each other on one communicator). On a full xGMI mesh a ring is bound by ONE link per
// direction per rank (busBW <= B_link) and the chain by one link (algBW <= B_link); the direct kernel uses
// all n-1 links. They exist for the reference's algorithm choice (C4's ring-vs-tree curve), not speed.
//
// Fold orders. Ring AllReduce: the reference's own partition (channel parts, loops of n chunks, the last loop
// re-cut, all_reduce.h:21-81; planned by enqueue.cc ringParts); chunk q of a loop starts at rank q+1 with
// pre(x_{q+1}) and each next rank folds red(pre(x_r), acc), ending at q — the reference's RING/SIMPLE order
// on the same channel count (oracle_all_reduce_ring_nccl). Ring ReduceScatter: block q folds from q+1.
// Chain AllReduce: the reference's intra-node tree with treeIntra = (0, 1, ..., n-1): leaf n-1 sends pre(x_{n-1}), rank k folds red(pre(x_k), acc) and the root 0 finishes (post) and broadcasts
// back down: order n-1, n-2, ..., 0 for every element (oracle_all_reduce_chain). Chain Reduce: the
// reference's ring reduce, root+1, ..., root (reduce.h:34-52).
#pragma once

namespace ncclamd {

enum PipeMode { MV_COPY = 0, MV_PRE = 1, MV_FOLD = 2, MV_FINAL = 3 };

// Wave 0 lanes i < n poll *ptr[i] >= val[i] (the direct kernel's waitAll over explicit flag words).
__device__ bool waitWords(const DevComm& dc, ChanState& st, const uint64_t* const* ptr, const uint64_t* val, int n,
                          bool ACQ) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const bool need = lane < n;
    uint64_t t0 = 0;
    uint32_t iter = 0;
    while (true) {
      bool ok = !need || loadFlag(ptr[lane]) >= val[lane];
      if (__all(ok)) break;
      if (iter == 0) t0 = clockTicks();
      __builtin_amdgcn_s_sleep(1);
      if ((++iter & 255) == 0) {
        bool bad = false;
        if (__hip_atomic_load(dc.abortFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          if (lane == 0) reportError(dc, DERR_ABORT);
          bad = true;
        } else if (__hip_atomic_load(dc.errorWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          bad = true;
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
    if (ACQ && lane == 0) __atomic_thread_fence(__ATOMIC_ACQUIRE);
    drainStores();
  }
  __syncthreads();
  return st.abort == 0;
}

// One hop's data movement, 16-byte packs when `aligned`:
//   MV_COPY  out = acc                      MV_PRE   out = pre(x)
//   MV_FOLD  out = red(pre(x), acc)         MV_FINAL out = post(red(pre(x), acc))
// written to dstLocal (nontemporal) and/or dstPush (write-through system scope, a peer's staging slot).
template <typename T, int OP, int MODE>
__device__ __forceinline__ void pipeMove(const Red<T, OP>& fn, const char* acc, const char* x, uint64_t nelem,
                                         char* dstLocal, char* dstPush, bool aligned) {
  constexpr int EPP = 16 / sizeof(T);
  constexpr int U = sizeof(T) == 1 ? 1 : 4;
  auto elem = [&](T av, T xv) -> T {
    if (MODE == MV_COPY) return av;
    if (MODE == MV_PRE) return fn.pre(xv);
    T r = fn.red(fn.pre(xv), av);
    return MODE == MV_FINAL ? fn.post(r) : r;
  };
  uint64_t npk = aligned ? nelem / EPP : 0;
  for (uint64_t base = threadIdx.x; base < npk; base += (uint64_t)U * kThreads) {
    PackU<T> av[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + (uint64_t)u * kThreads;
      if (i >= npk) continue;
      if (MODE != MV_PRE) av[u].v = __builtin_nontemporal_load((const u32x4*)acc + i);
      if (MODE != MV_COPY) xv[u].v = __builtin_nontemporal_load((const u32x4*)x + i);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = base + (uint64_t)u * kThreads;
      if (i >= npk) continue;
      PackU<T> o;
      if (MODE == MV_COPY) o = av[u];
      else
#pragma unroll
        for (int e = 0; e < EPP; e++) o.e[e] = elem(av[u].e[e], xv[u].e[e]);
      if (dstLocal) __builtin_nontemporal_store(o.v, (u32x4*)dstLocal + i);
      if (dstPush) {
        if (NCCL_AMD_BUFFER_STORES) storeRemoteAt(remoteRsrc(dstPush), (uint32_t)(i * 16), o.v);
        else storeRemote((u32x4*)dstPush + i, o.v);
      }
    }
  }
  for (uint64_t t = npk * EPP + threadIdx.x; t < nelem; t += kThreads) {  // tail / unaligned
    const T av = MODE == MV_PRE ? T{} : ((const T*)acc)[t];
    const T xv = MODE == MV_COPY ? T{} : ((const T*)x)[t];
    const T o = elem(av, xv);
    if (dstLocal) ((T*)dstLocal)[t] = o;
    if (dstPush) storeRemoteElt((T*)dstPush + t, o);
  }
}

struct PipeShared {
  ChanState st;
  const uint64_t* waitPtr[2];
  uint64_t waitVal[2];
  uint64_t* sigPtr[2];
  uint64_t sigVal[2];
  int nWait;
};

template <typename T, int OP>
struct Pipe {
  const CollArgs& a;
  const DevComm& dc;
  PipeShared& sh;
  const Red<T, OP>& fn;
  int c, me, n, nSlots;
  bool aligned;
  static constexpr uint64_t ts = sizeof(T);

  __device__ uint64_t& ctr(int k, int r) const { return sh.st.ctr[k][r]; }

  // One hop on a connection kind (STG_RS: the ring / the chain's way up; STG_AG: the chain's way down):
  // receive a slot from `from` (or -1), send a slot to `to` (or -1). x: this rank's input slice; out: its
  // output slice (either may be null as MODE requires).
  template <int MODE>
  __device__ bool hop(int kind, int from, int to, const char* x, char* out, uint64_t nelem) {
    const int ckSend = kind == STG_RS ? CTR_SEND_RS : CTR_SEND_AG, ckRecv = kind == STG_RS ? CTR_RECV_RS : CTR_RECV_AG;
    const int fReady = kind == STG_RS ? FLG_RS_READY : FLG_AG_READY, fAck = kind == STG_RS ? FLG_RS_ACK : FLG_AG_ACK;
    const int tid = threadIdx.x;
    const uint64_t* myFlags = dc.flags[me] + flagIndex(c, 0, 0);
    if (tid == 0) {
      int nw = 0;
      if (from >= 0) {
        sh.waitPtr[nw] = myFlags + flagIndex(0, fReady, from);
        sh.waitVal[nw++] = ctr(ckRecv, from) + 1;
      }
      const uint64_t s = to >= 0 ? ctr(ckSend, to) : 0;
      if (to >= 0 && s + 1 > (uint64_t)nSlots) {  // the slot we are about to overwrite must be consumed
        sh.waitPtr[nw] = myFlags + flagIndex(0, fAck, to);
        sh.waitVal[nw++] = s + 1 - nSlots;
      }
      sh.nWait = nw;
    }
    __syncthreads();
    if (!waitWords(dc, sh.st, sh.waitPtr, sh.waitVal, sh.nWait, from >= 0)) return false;
    const char* acc = from >= 0 ? dc.staging[me] + stagingOffset(dc, c, kind, (int)(ctr(ckRecv, from) % nSlots), from)
                                : x;  // MV_COPY from my own input (a chain's root or a ring's first AG hop)
    char* push = to >= 0 ? dc.staging[to] + stagingOffset(dc, c, kind, (int)(ctr(ckSend, to) % nSlots), me) : nullptr;
    pipeMove<T, OP, MODE>(fn, acc, x, nelem, out, push, aligned);
    if (tid == 0) {
      sh.sigPtr[0] = to >= 0 ? dc.flags[to] + flagIndex(c, fReady, me) : nullptr;  // data ready
      sh.sigVal[0] = to >= 0 ? ctr(ckSend, to) + 1 : 0;
      sh.sigPtr[1] = from >= 0 ? dc.flags[from] + flagIndex(c, fAck, me) : nullptr;  // slot consumed
      sh.sigVal[1] = from >= 0 ? ctr(ckRecv, from) + 1 : 0;
    }
    __syncthreads();
    // every pushed byte is a write-through system-scope store, drained in signalAll before the flag
    signalAll(sh.sigPtr, sh.sigVal, 2, (a.protoFlags & 8) == 0);
    if (tid == 0) {
      if (to >= 0) ctr(ckSend, to)++;
      if (from >= 0) ctr(ckRecv, from)++;
    }
    __syncthreads();
    return true;
  }
};

template <typename T, int OP, int KIND>
__global__ void __launch_bounds__(kThreads) kCoResident pipeKernel(CollArgs a) {
  __shared__ PipeShared sh;
  const DevComm& dc = *a.comm;
  const int tid = threadIdx.x, c = blockIdx.x, me = dc.rank, n = dc.nRanks;
  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    sh.st.ctr[k][r] = dc.counters[ctrIndex(c, k, r)];
  }
  if (tid == 0) sh.st.abort = 0;
  __syncthreads();
  uint64_t opArg = a.redArg;
  if (a.redArgPtr) {
    opArg = 0;
    __builtin_memcpy(&opArg, a.redArgPtr, sizeof(T));
  }
  const Red<T, OP> fn(opArg);
  Pipe<T, OP> p{a, dc, sh, fn, c, me, n, dc.nSlots, a.aligned != 0};
  constexpr uint64_t ts = sizeof(T);
  const char* in = (const char*)a.sendbuff;
  char* outb = (char*)a.recvbuff;
  const int next = (me + 1) % n, prev = (me + n - 1) % n;
  bool ok = true;
  if (KIND == PIPE_RING_AR) {
    // The reference's runRing over its own partition (all_reduce.h:21-81): this channel's part
    // (ncclCollCbdPart, device.h:337-361: the first channel takes cbdLo elements, the middle ones `part`, the
    // last cbdHi), walked in loops of n chunks of a.chunk elements; the last loop re-cuts the chunk to
    // alignUp(divUp(rem, n), 16 / sizeof(T)) (:38). Chunk q of a loop starts at rank q+1 and is finalised by
    // rank q, so every element folds exactly as in the reference's RING/SIMPLE AllReduce on the same number of
    // channels. A chunk moves through the staging slots in slices of a.slice elements; every rank walks the
    // same loops and slices (the counts are shared), so the hops pair up. a.refSub workgroups share one part:
    // workgroup c serves part c / refSub and moves sub-chunk c % refSub of every chunk (CollArgs::refSub) — the
    // ring position that finalises an element, hence its fold order, does not depend on the workgroup.
    constexpr uint64_t EPP = 16 / ts;
    const uint32_t G = a.refSub, sub = (uint32_t)c % G;
    const int nParts = (int)(gridDim.x / G), k = (int)((uint32_t)c / G);
    uint64_t pOff, pCnt;
    if (k == 0) pOff = 0, pCnt = a.cbdLo;
    else if (k == nParts - 1) pOff = a.cbdLo + (uint64_t)(nParts - 2) * a.part, pCnt = a.cbdHi;
    else pOff = a.cbdLo + (uint64_t)(k - 1) * a.part, pCnt = a.part;
    const uint64_t loopCount = (uint64_t)n * a.chunk;
    for (uint64_t eo = 0; ok && eo < pCnt; eo += loopCount) {
      const uint64_t rem = pCnt - eo;
      const uint64_t ck = rem < loopCount ? ((rem + n - 1) / n + EPP - 1) / EPP * EPP : a.chunk;
      const uint64_t sc = ((ck + G - 1) / G + EPP - 1) / EPP * EPP;  // sub-chunk length
      const uint64_t scLo = min((uint64_t)sub * sc, ck);
      const char* inL = in + (pOff + eo) * ts;
      char* outL = outb + (pOff + eo) * ts;
      const uint64_t nSub = (min(scLo + sc, ck) - scLo + a.slice - 1) / a.slice;
      for (uint64_t s = 0; ok && s < nSub; s++) {
        uint64_t lo, hi;
        auto sl = [&](int q) {  // slice s of my sub-chunk of chunk q (empty past the loop's end)
          const uint64_t b = (uint64_t)q * ck, len = b >= rem ? 0 : min(ck, rem - b);
          const uint64_t sLo = min((uint64_t)sub * sc, len), sHi = min(sLo + sc, len);
          lo = min(sLo + s * a.slice, sHi);
          hi = min(lo + a.slice, sHi);
        };
        auto at = [&](int q) { return ((uint64_t)q * ck + lo) * ts; };
        int q = prev;  // step 0: send chunk ringIx - 1
        sl(q);
        ok = p.template hop<MV_PRE>(STG_RS, -1, next, inL + at(q), nullptr, hi - lo);
        for (int j = 2; ok && j < n; j++) {  // n-2 x recvReduceSend
          q = (me + n - j) % n;
          sl(q);
          ok = p.template hop<MV_FOLD>(STG_RS, prev, next, inL + at(q), nullptr, hi - lo);
        }
        if (!ok) break;
        sl(me);  // recvReduceCopySend: the final value of my chunk
        ok = p.template hop<MV_FINAL>(STG_RS, prev, next, inL + at(me), outL + at(me), hi - lo);
        for (int j = 1; ok && j < n - 1; j++) {  // n-2 x recvCopySend
          q = (me + n - j) % n;
          sl(q);
          ok = p.template hop<MV_COPY>(STG_RS, prev, next, nullptr, outL + at(q), hi - lo);
        }
        if (!ok) break;
        q = next;  // recv: the chunk next finalised
        sl(q);
        ok = p.template hop<MV_COPY>(STG_RS, prev, -1, nullptr, outL + at(q), hi - lo);
      }
    }
  } else if (KIND == PIPE_RING_RS || KIND == PIPE_RING_AG) {
    // Reduce-scatter: block q (a.chunk = recvcount elements) is rank q's output and folds from q+1 whatever the
    // partition; AllGather: block q of the output is rank q's input. Each channel takes a part of every block.
    for (int s = 0; ok && s < a.nSteps; s++) {
      uint64_t lo, hi;
      auto sl = [&](int) { sliceRange(a, c, s, a.chunk, lo, hi); };
      if (KIND == PIPE_RING_RS) {
        int q = prev;  // step 0 of the reference's ring: send chunk ringIx-1
        sl(q);
        ok = p.template hop<MV_PRE>(STG_RS, -1, next, in + ((uint64_t)q * a.chunk + lo) * ts, nullptr, hi - lo);
        for (int j = 2; ok && j < n; j++) {  // n-2 x recvReduceSend
          q = (me + n - j) % n;
          sl(q);
          ok = p.template hop<MV_FOLD>(STG_RS, prev, next, in + ((uint64_t)q * a.chunk + lo) * ts, nullptr, hi - lo);
        }
        if (!ok) break;
        sl(me);  // recvReduceCopy: the final value of my block
        ok = p.template hop<MV_FINAL>(STG_RS, prev, -1, in + ((uint64_t)me * a.chunk + lo) * ts, outb + lo * ts,
                                      hi - lo);
      } else {
        sl(me);  // AllGather step 0: my input to my output block and to next
        char* o = outb + ((uint64_t)me * a.chunk + lo) * ts;
        const char* x = in + lo * ts;
        ok = p.template hop<MV_COPY>(STG_RS, -1, next, x, o == x ? nullptr : o, hi - lo);
      }
      if (KIND == PIPE_RING_RS) continue;
      for (int j = 1; ok && j < n - 1; j++) {  // n-2 x recvCopySend
        const int q = (me + n - j) % n;
        sl(q);
        ok = p.template hop<MV_COPY>(STG_RS, prev, next, nullptr, outb + ((uint64_t)q * a.chunk + lo) * ts, hi - lo);
      }
      if (!ok) break;
      const int q = next;  // recv: the block next finalised
      sl(q);
      ok = p.template hop<MV_COPY>(STG_RS, prev, -1, nullptr, outb + ((uint64_t)q * a.chunk + lo) * ts, hi - lo);
    }
  } else {
    // chain positions 0..n-1 (0 = leaf, n-1 = root): AllReduce = the reference's intra-node tree with root 0
    // and leaf n-1 (position p is rank n-1-p); Reduce = the reference's ring reduce root+1 -> ... -> root
    const bool ar = KIND == PIPE_CHAIN_AR;
    auto rankAt = [&](int pos) { return ar ? n - 1 - pos : (a.root + 1 + pos) % n; };
    const int pos = ar ? n - 1 - me : (me + n - a.root - 1) % n;
    const int down = pos > 0 ? rankAt(pos - 1) : -1, up = pos < n - 1 ? rankAt(pos + 1) : -1;
    for (int s = 0; ok && s < a.nSteps; s++) {  // reduce up
      uint64_t lo, hi;
      sliceRange(a, c, s, a.count, lo, hi);
      const char* x = in + lo * ts;
      if (pos == 0) ok = p.template hop<MV_PRE>(STG_RS, -1, up, x, nullptr, hi - lo);
      else if (up >= 0) ok = p.template hop<MV_FOLD>(STG_RS, down, up, x, nullptr, hi - lo);
      else ok = p.template hop<MV_FINAL>(STG_RS, down, -1, x, outb + lo * ts, hi - lo);
    }
    for (int s = 0; ar && ok && s < a.nSteps; s++) {  // broadcast down from the root
      uint64_t lo, hi;
      sliceRange(a, c, s, a.count, lo, hi);
      char* o = outb + lo * ts;
      if (up < 0) ok = p.template hop<MV_COPY>(STG_AG, -1, down, o, nullptr, hi - lo);
      else ok = p.template hop<MV_COPY>(STG_AG, up, down, nullptr, o, hi - lo);
    }
  }
  __syncthreads();
  if (tid < CTR_KINDS * NCCL_AMD_MAX_RANKS) {
    int k = tid / NCCL_AMD_MAX_RANKS, r = tid % NCCL_AMD_MAX_RANKS;
    dc.counters[ctrIndex(c, k, r)] = sh.st.ctr[k][r];
  }
}

}  // namespace ncclamd
