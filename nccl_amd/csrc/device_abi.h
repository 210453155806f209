// device_abi.h — data layout shared by the host runtime and the gfx950 kernels.
//
// HBM layout per rank (all offsets in bytes, every region 16-byte aligned):
//
//   staging  (hipExtMallocWithFlags(..., hipDeviceMallocUncached), exported by HIP IPC)
//     [channel c < maxChannels][kind k < 2 (RS, AG)][slot s < nSlots][from < nRanks][slotBytes]
//     Written ONLY by peer `from` over xGMI (remote write-through stores); read ONLY by the owner.
//
//   flags    (uncached, exported by HIP IPC)
//     uint64 [channel][flag kind < 4][from < NCCL_AMD_MAX_RANKS]
//       RS_READY[c][from]  = number of RS slices `from` has written into my staging (monotonic)
//       RS_ACK[c][from]    = number of my RS slices `from` has consumed from ITS staging
//       AG_READY / AG_ACK  = the same for the all-gather direction
//       SYM_ENTER / SYM_MID / SYM_DONE[c][from] = epoch of the last symmetric (window) collective in
//                          which `from` entered / published its reduced block / finished reading peers
//       REG_SEND / REG_RECV[c][from] = `from`'s registered send / recv buffer as mapped in MY address space,
//                          stored before its SYM_ENTER (zero-copy collectives on ncclCommRegister buffers)
//     A word is written by exactly one remote rank and polled only by its owner.
//
//   LL lines (same uncached allocation as the flags, at DevComm::llOffset; reference prims_ll.h:108-158)
//     [channel < llChannels][parity < 2][from < nRanks][llBytes]: 16-byte lines {data32, flag32, data32,
//     flag32} written by `from` with one write-through store; the flag is the channel's LL epoch, so the
//     reader needs neither a flag word nor a fence. Parity = epoch & 1 (double buffering).
//
//   LL64 lines (the LL128-class protocol, at DevComm::ll64Offset; reference prims_ll128.h): same geometry,
//     64-byte lines = 4 lanes x 16 bytes = 56 bytes of payload + the 64-bit epoch flag in the last 8 bytes.
//     64 bytes, not the reference's 128: on MI355X a 128-byte line written by one wave-instruction is
//     observed torn, 64-byte segments are not (tests/native/store_atomicity_probe).
//     A separate area, so stale LL64 payload can never alias an LL flag position and vice versa.
//
//   counters (plain device memory, local)
//     uint64 [channel][ctr kind < 5 (sendRS, recvRS, sendAG, recvAG, sym)][peer < NCCL_AMD_MAX_RANKS]
//     Per-connection step counters (reference: conn->step, src/device/prims_simple.h:100-173),
//     kept in device memory so a captured hipGraph replays correctly.
#pragma once
#include <stdint.h>

#define NCCL_AMD_MAX_RANKS 16
#define NCCL_AMD_MAX_CHANNELS 256

namespace ncclamd {

enum StagingKind { STG_RS = 0, STG_AG = 1, STG_KINDS = 2 };
// FLG_PULL_READY / FLG_PULL_ACK and CTR_PULL_PUB / CTR_PULL_GOT: the AG-pull gather (kernels.h
// Channel::agPull) publishes ONE copy per step that every peer reads, so it keeps its own sequence (the
// per-pair AG counters diverge once a Reduce has pushed to its root only).
// FLG_REG_SEND / FLG_REG_RECV: the device-side pointer exchange of registered (ncclCommRegister) buffers —
// before its ENTER signal, rank `from` stores its send / recv buffer AS MAPPED IN THIS PROCESS into these
// words of the same channel (reference: the ptrExchange slots of prims_simple.h:748-846).
enum FlagKind {
  FLG_RS_READY = 0, FLG_RS_ACK = 1, FLG_AG_READY = 2, FLG_AG_ACK = 3,
  FLG_SYM_ENTER = 4, FLG_SYM_MID = 5, FLG_SYM_DONE = 6, FLG_PULL_READY = 7, FLG_PULL_ACK = 8,
  FLG_REG_SEND = 9, FLG_REG_RECV = 10, FLG_KINDS = 11
};
enum CtrKind {
  CTR_SEND_RS = 0, CTR_RECV_RS = 1, CTR_SEND_AG = 2, CTR_RECV_AG = 3, CTR_SYM = 4, CTR_LL = 5,
  CTR_PULL_PUB = 6, CTR_PULL_GOT = 7, CTR_KINDS = 8
};

// Ring / chain kernels (pipe.h; NCCL_ALGO=RING / TREE)
enum PipeKind { PIPE_RING_AR = 0, PIPE_RING_RS = 1, PIPE_RING_AG = 2, PIPE_CHAIN_AR = 3, PIPE_CHAIN_REDUCE = 4 };

// Device reduction kinds (reference ncclDevRedOp_t subset, src/include/device.h)
enum DevRedOp { DEV_SUM = 0, DEV_PROD = 1, DEV_MINMAX = 2, DEV_PREMULSUM = 3, DEV_SUMPOSTDIV = 4, DEV_NUMOPS = 5 };

// Error codes written by a kernel into the host-visible error word.
// DERR_MISMATCH: a peer ran another kernel kind for the same collective (registered zero-copy vs staged; the
// wait probe in kernels.h waitAll), reported instead of waiting for the spin timeout.
enum DevError { DERR_NONE = 0, DERR_TIMEOUT = 1, DERR_ABORT = 2, DERR_MISMATCH = 3 };

struct DevComm {
  int rank;
  int nRanks;
  int nSlots;
  int maxChannels;
  uint64_t slotBytes;
  uint64_t timeoutTicks;  // s_memrealtime ticks (100 MHz) before a spin gives up
  char* staging[NCCL_AMD_MAX_RANKS];     // every rank's staging base as mapped here
  uint64_t* flags[NCCL_AMD_MAX_RANKS];   // every rank's flag block as mapped here
  uint64_t* counters;                    // local step counters
  uint64_t llOffset;                     // LL line area inside every rank's flag allocation
  uint64_t llBytes;                      // line bytes per (channel, parity, sender)
  uint64_t ll64Offset;                   // LL64 line area (same geometry as the LL area)
  int llChannels;
  uint32_t* abortFlag;                   // host-pinned; nonzero = abort
  uint32_t* errorWord;                   // host-pinned; first DevError recorded
};

// Kernel argument block (passed by value, < 4 KiB like the reference's ncclDevKernelArgs4K,
// src/device/common.h:435-449).
struct CollArgs {
  const void* sendbuff;
  void* recvbuff;
  const DevComm* comm;
  uint64_t count;      // AR/Reduce: elements; RS: recvcount; AG: sendcount (bytes for AG)
  uint64_t chunk;      // elements per rank block (AR: alignUp(divUp(count,n),EPP); RS/AG: count)
  uint64_t part;       // elements per channel within a rank block
  uint64_t slice;      // elements per pipeline step (per peer)
  uint64_t redArg;     // scalar / xormask / divisor bits
  const void* redArgPtr;  // device scalar (PreMulSum with ncclScalarDevice), else nullptr
  int nSteps;
  int root;
  int aligned;         // send/recv base pointers are 16-byte aligned
  int protoFlags;      // NCCL_AMD_PROTO_FLAGS diagnostics (kernels.h collKernel)
  // Ring AllReduce (PIPE_RING_AR) and the reference-order direct AllReduce (COLL_ARREF) in the reference's
  // partition: channel parts lo / mid (= part) / hi (ncclCollCbdPart, reference src/include/device.h:337-361),
  // each walked in loops of n chunks of `chunk` elements (all_reduce.h:21-38). Unused by every other kernel.
  uint64_t cbdLo, cbdHi;
  // ... and refSub workgroups per reference channel part: workgroup c serves part c / refSub and, inside every
  // chunk of that part, the sub-chunk c % refSub (an element's fold order depends only on its loop and chunk,
  // never on which workgroup moves it), so the reference's channel count and this launch's parallelism are
  // independent.
  uint32_t refSub;
  uint32_t refPad;
};

// Staged batch: up to kMaxCollBatch ops of one group with the same collective, type and op (and the same
// one-shot / direct choice) in ONE collBatchKernel launch; op k runs on channels chOff[k] .. + nch[k] - 1.
constexpr int kMaxCollBatch = 8;
struct CollBatchArgs {
  CollArgs op[kMaxCollBatch];
  int chOff[kMaxCollBatch];
  int nch[kMaxCollBatch];
  int nOps;
};

// LL batch: up to kMaxLLBatch small ops of one group (same comm, stream, type and op; any of AllReduce,
// ReduceScatter, AllGather, Reduce) run by ONE launch (reference: ops of a group aggregated into one kernel
// plan, enqueue.cc:405-470).
constexpr int kMaxLLBatch = 32;
enum LLColl { LL_AR = 0, LL_RS = 1, LL_AG = 2, LL_REDUCE = 3 };
enum LLProto { LLP_LL = 0, LLP_LL64 = 1 };
constexpr int kLL64Payload = 56;  // payload bytes per 64-byte LL64 line
struct LLOp {
  const void* send;
  void* recv;
  uint64_t count;  // elements (AllReduce: of the buffer; ReduceScatter / AllGather: of one rank block)
  uint64_t chunk;  // elements per rank block (fold order of each element's owner)
  uint64_t part;   // 8-byte payloads per channel
  int nch;         // channels this op uses
  int chOff;       // first channel (batches spread their ops over the LL channels)
  int coll;        // LLColl
  int root;        // LL_REDUCE: the rank that folds and stores (the others send and poll only)
  int proto;       // LLProto: LL (part = 8-byte payloads) or LL64 (part = 64-byte lines of 56 payload bytes)
};
// The kernel arguments hold room for K ops: a lone op launches with K = 1 (88 bytes of kernel arguments
// instead of 1.8 KiB; the host issue cost of a launch grows with its argument bytes, about 3 us at 64 B
// vs 6.5 us at 2 KiB on the MI355X box, scripts/launch_probe.hip).
// A batch (K > 1) also carries, per LL channel (at most 32), the bit mask of the ops that run on it: a work-group
// reads ONE word of the argument block to find its ops, instead of every op's channel range (each op descriptor
// its own line of the argument block, and every work-group of the launch reading them all).
constexpr int kMaxLLChannels = 32;
template <int K>
struct LLArgs {
  const DevComm* comm;
  uint64_t* counters;  // comm->counters (device): the channels' LL epochs load beside the DevComm, not after it
  uint64_t redArg;
  const void* redArgPtr;
  int nOps;
  uint32_t chMask[K > 1 ? kMaxLLChannels : 1];  // bit k: op k runs on this channel (K > 1 only)
  LLOp ops[K];
};
static_assert(kMaxLLBatch <= 32, "LLArgs::chMask holds one bit per op");
using LLBatchArgs = LLArgs<kMaxLLBatch>;

// Symmetric (window) collective arguments: every rank's buffers as mapped in this process (reference
// ncclSymPtr::peerPtr, src/device/symmetric/kernel.cuh), so peers are read and written directly.
// regMode (buffers registered with ncclCommRegister, reference src/register/coll_reg.cc:326-395): the host
// knows only where ITS OWN buffers are mapped in every peer, so send[r] / recv[r] (r != rank) hold MY buffers
// as mapped in rank r; the kernel hands them to rank r through r's FLG_REG_SEND / FLG_REG_RECV words and reads
// the peers' buffers from its own words after the ENTER handshake (the reference's ptrExchange,
// prims_simple.h:748-846). `aligned` then carries only the count condition: pointer alignment of every
// rank's buffers is decided in the kernel, from the exchanged pointers, identically on every rank.
struct SymArgs {
  const DevComm* comm;
  const char* send[NCCL_AMD_MAX_RANKS];  // rank r's sendbuff (regMode: my sendbuff as mapped in rank r)
  char* recv[NCCL_AMD_MAX_RANKS];        // rank r's recvbuff (regMode: my recvbuff as mapped in rank r)
  uint64_t count;      // AR: elements; RS: recvcount; AG: sendcount
  uint64_t chunk;      // elements per rank block
  uint64_t part;       // elements per channel (AR two-shot / RS / AG: within a block; one-shot: of the buffer)
  uint64_t redArg;
  const void* redArgPtr;
  int aligned;
  int wtPublish;       // bytes peers read (AR fold result, AG own block) stored write-through: no L2 write-back
  int regMode;         // buffers registered with ncclCommRegister: device-side pointer exchange (above)
  int relFence;        // publish with a system release fence even after write-through stores (across devices)
};

// Mapping check at communicator init (mapcheck.cc, kernels.hip mapCheckKernel): the words this rank stores into
// peer p's staging slab (w[p][0]) and flag block (w[p][1]) through its mappings of them.
struct MapCheckArgs {
  uint64_t w[NCCL_AMD_MAX_RANKS][2][2];
  uint64_t probeOff;  // the check area inside every rank's flag allocation (same offset everywhere)
  int skip;           // tests (NCCL_AMD_MAPCHECK_FAULT): no stores, as a mapping that drops them
};

__host__ __device__ inline uint64_t stagingOffset(const DevComm& dc, int c, int kind, int slot, int from) {
  return ((((uint64_t)c * STG_KINDS + kind) * dc.nSlots + slot) * dc.nRanks + from) * dc.slotBytes;
}
__host__ __device__ inline uint64_t llLineOffset(const DevComm& dc, int c, int parity, int from) {
  return dc.llOffset + (((uint64_t)c * 2 + parity) * dc.nRanks + from) * dc.llBytes;
}
__host__ __device__ inline uint64_t ll64LineOffset(const DevComm& dc, int c, int parity, int from) {
  return dc.ll64Offset + (((uint64_t)c * 2 + parity) * dc.nRanks + from) * dc.llBytes;
}
__host__ __device__ inline uint64_t flagIndex(int c, int kind, int from) {
  return ((uint64_t)c * FLG_KINDS + kind) * NCCL_AMD_MAX_RANKS + from;
}
__host__ __device__ inline uint64_t ctrIndex(int c, int kind, int peer) {
  return ((uint64_t)c * CTR_KINDS + kind) * NCCL_AMD_MAX_RANKS + peer;
}
// The k-th peer (k = 1 .. n-1) that channel c of rank `me` visits in a workgroup-wide multi-peer loop: the
// staged scatter's pushes, the pull gather's reads, the zero-copy kernels' reads. Rotated by channel: with one
// order on every channel, all of a rank's channels would sit on the SAME peer's xGMI link at step position k;
// rotated, any n-1 consecutive channels put position k on all n-1 peers once (a Latin square), and for a fixed
// (c, k) the ranks' choices are a shift, so every peer is also the source / target of exactly one rank.
// Data placement and fold order never depend on it (tests/native/plan_test `peers`).
__host__ __device__ inline int chanPeer(int me, int n, int c, int k) {
  return (me + 1 + (k - 1 + c) % (n - 1)) % n;
}

}  // namespace ncclamd
