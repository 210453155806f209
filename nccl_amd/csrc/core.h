// core.h — internal definitions of the MI355X reduction engine (host side).
//
// Layer map (reference SURVEY.md §1): L7 public API (api.cc) → L5 enqueue/group (enqueue.cc, group.cc)
// → L6 device kernels (kernels.hip) over L3 peer-mapped staging (transport.cc) set up by
// L4 init (init.cc) using the L1 TCP bootstrap (bootstrap.cc). L0 = debug.cc / param.cc.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <functional>
#include <memory>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nccl.h"
#include "device_abi.h"

#define NCCL_EXPORT extern "C" __attribute__((visibility("default")))

namespace ncclamd {

// ---------------------------------------------------------------- logging (reference src/debug.cc)
enum LogLevel { LOG_NONE = 0, LOG_VERSION = 1, LOG_WARN = 2, LOG_INFO = 3, LOG_ABORT = 4, LOG_TRACE = 5 };
void logInit();
extern int gLogLevel;
void logMessage(int level, const char* file, int line, const char* fmt, ...) __attribute__((format(printf, 4, 5)));
void setLastError(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* lastError();

#define WARN(...) ::ncclamd::logMessage(::ncclamd::LOG_WARN, __FILE__, __LINE__, __VA_ARGS__)
#define INFO(...)                                                                         \
  do {                                                                                    \
    if (::ncclamd::gLogLevel >= ::ncclamd::LOG_INFO)                                      \
      ::ncclamd::logMessage(::ncclamd::LOG_INFO, __FILE__, __LINE__, __VA_ARGS__);        \
  } while (0)
#define TRACE(...)                                                                        \
  do {                                                                                    \
    if (::ncclamd::gLogLevel >= ::ncclamd::LOG_TRACE)                                     \
      ::ncclamd::logMessage(::ncclamd::LOG_TRACE, __FILE__, __LINE__, __VA_ARGS__);       \
  } while (0)

#define NCCLCHECK(call)                                   \
  do {                                                    \
    ncclResult_t _r = (call);                             \
    if (_r != ncclSuccess && _r != ncclInProgress) {      \
      INFO("%s:%d -> %d", __FILE__, __LINE__, (int)_r);   \
      return _r;                                          \
    }                                                     \
  } while (0)

#define HIPCHECK(call)                                                           \
  do {                                                                           \
    hipError_t _e = (call);                                                      \
    if (_e != hipSuccess) {                                                      \
      WARN("HIP failure '%s' at %s", hipGetErrorString(_e), #call);              \
      return ncclUnhandledCudaError;                                             \
    }                                                                            \
  } while (0)

#define SYSCHECK(cond, what)                                                     \
  do {                                                                           \
    if (!(cond)) {                                                               \
      WARN("system error in %s: %s", what, strerror(errno));                     \
      return ncclSystemError;                                                    \
    }                                                                            \
  } while (0)

// roctx range around an API call (NCCL_AMD_ROCTX=1; reference NVTX ranges, src/collectives.cc:134,170)
extern int gRoctx;
struct RoctxRange {
  bool on = false;
  void push(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
  ~RoctxRange();
};
// the arguments are evaluated only when ranges are on
#define ROCTX_RANGE(...)                  \
  ::ncclamd::RoctxRange _roctxRange;      \
  if (::ncclamd::gRoctx) _roctxRange.push(__VA_ARGS__)

// ---------------------------------------------------------------- params (reference src/misc/param.cc)
int64_t paramInt(const char* name, int64_t deflt);
const char* paramStr(const char* name);  // nullptr when unset

// ---------------------------------------------------------------- bootstrap (reference src/bootstrap.cc)
struct Bootstrap;
struct LocalClique;
ncclResult_t bootstrapGetUniqueId(ncclUniqueId* id);
ncclResult_t bootstrapInit(const ncclUniqueId* id, int rank, int nranks, Bootstrap** out);
ncclResult_t bootstrapRelease(const ncclUniqueId* id);  // tell an unused root to exit (InitRankScalable)
ncclResult_t bootstrapReleaseUnused(const ncclUniqueId* ids, int nId, int rank, int nranks);  // this rank's share
ncclResult_t bootstrapAllGather(Bootstrap* b, void* data, size_t bytesPerRank);
ncclResult_t bootstrapBarrier(Bootstrap* b);
void bootstrapClose(Bootstrap* b);
std::shared_ptr<LocalClique> cliqueCreate(int nranks);
ncclResult_t cliqueAllGather(LocalClique* c, int rank, void* data, size_t bytesPerRank);

// ---------------------------------------------------------------- communicator (reference src/include/comm.h)
constexpr uint64_t kCommMagic = 0x4d493335584e4343ull;  // "MI35XNCC"

// ---------------------------------------------------------------- cross-process memory (ipc.cc)
// An exported allocation as a peer sees it: the dma-buf fd server and key to fetch it from (reference: cuMem
// POSIX fd handles, src/transport/p2p.cc:220-325), or a legacy hipIpc handle (NCCL_AMD_IPC=legacy).
struct IpcDesc {
  uint64_t key;
  uint64_t size;
  char server[40];  // abstract UNIX socket name of the exporter's fd server
  int legacy;       // NCCL_AMD_IPC=legacy: handle only
  int hasHandle;    // dma-buf export that also carries a hipIpc handle (import fallback, ipc.cc)
  hipIpcMemHandle_t handle;
};
struct IpcImport {  // one mapping of a peer's allocation in this process
  void* ptr;
  void* ext;  // hipExternalMemory_t
  int fd;
  int legacy;
  uint64_t fdDev, fdIno;  // identity of fd at import (ipcRelease closes it only if it still names that file)
  uint64_t size;          // bytes mapped (the pending-release account, ipc.cc)
};
struct FdServer;
bool ipcLegacy();
const char* ipcServerName(const ncclComm* comm);  // "" without an fd server
// Release peers' mappings whose owner deregistered them (ipc.cc): called on the caller's thread at the blocking entry
// points (init, finalize, destroy, (de)registration); a no-op unless a RELEASE arrived.
void ipcDrainReleases();
// The same on the collective path (ipc.cc): mappings whose owner released them, unmapped without waiting for the device
void ipcProgressReleases();
// after each kernel launch of a multi-process communicator (outside captures): the stream's tail event (ipc.cc)
void ipcNoteLaunch(hipStream_t stream, int device);
// none of this library's kernels in flight in this process (the streams ipcNoteLaunch tracks are idle)
bool ipcLibraryIdle();
// Held around this library's device allocations, imports and releases (ipc.cc gMapMu): no allocation of ours can
// interleave with a mapping being torn down on another thread (a non-blocking init runs on its own thread).
std::mutex& ipcMapMutex();
struct HipRuntimeInfo {
  int version;    // hipRuntimeGetVersion of the runtime bound in this process
  int driver;     // hipDriverGetVersion
  char path[256]; // the libamdhip64 it lives in (dladdr)
};
const HipRuntimeInfo& hipRuntimeInfo();
// may an allocation of `size` be shared by hipIpc handle on this runtime? (requested: NCCL_AMD_IPC=legacy)
bool ipcLegacyAllowed(int runtimeVersion, size_t size, bool requested);
ncclResult_t ipcServerStart(ncclComm* comm);
void ipcServerStop(ncclComm* comm);
ncclResult_t ipcExport(ncclComm* comm, void* base, size_t size, IpcDesc* d);
hipError_t ipcExportDmaBuf(void* base, size_t size, int* fd, int attempts = 5);  // under gMapMu (ipc.cc)
bool ipcAdmitExport(int fd, void* base, size_t size);  // its stale-export checks (ipc.cc; CPU-tested)
void ipcUnexport(ncclComm* comm, const IpcDesc& d);
ncclResult_t ipcPublish(ncclComm* comm, int fd, size_t size, IpcDesc* d);  // serve an fd (owned) under a new key
ncclResult_t ipcFetchFd(const IpcDesc& d, int* fd);  // an exporter's fd for d, over its fd server (bounded)
ncclResult_t ipcImport(const IpcDesc& d, IpcImport* out);
ncclResult_t ipcImportHandle(const IpcDesc& d, IpcImport* out);  // the hipIpc handle only (d.hasHandle or d.legacy)
void ipcRelease(IpcImport* m);
// Registered buffers (register.cc): ask the fd server `server` (a peer's) to map the dma-buf `fd` (sent along,
// the caller keeps its copy) on its device on behalf of `rank`, remembered under `tag`; *addr = where it
// landed in the peer's process. Release drops that mapping (best effort: a peer already gone released it).
ncclResult_t ipcRemoteImport(const char* server, int rank, uint64_t tag, int fd, uint64_t size, uint64_t* addr);
// the same with a hipIpc handle of the allocation instead of a dma-buf fd (the owner's export was refused)
ncclResult_t ipcRemoteImportHandle(const char* server, int rank, uint64_t tag, const hipIpcMemHandle_t& h, uint64_t size,
                                   uint64_t* addr);
void ipcRemoteRelease(const char* server, int rank, uint64_t tag);
uint64_t ipcNewTag();

struct PeerInfo {  // exchanged once at init (reference: struct ncclPeerInfo, src/init.cc:1035-1037)
  int rank;
  int device;
  int pid;
  uint64_t hostHash;
  char busId[32];
  int numCUs;
  IpcDesc stagingDesc;  // other processes import these
  IpcDesc flagsDesc;
  uint64_t stagingPtr;  // raw pointers, valid only inside the same process
  uint64_t flagsPtr;
  // this rank's fd server (ipc.cc), published on its own: a slab exported by the hipIpc fallback carries no server
  // name in its descriptor, yet the server still maps peers' registered buffers (register.cc)
  char fdServer[40];
};

struct UserRedOp {  // ncclRedOpCreatePreMulSum state (reference src/enqueue.cc:2560-2576)
  bool used;
  ncclDataType_t datatype;
  int devOp;
  uint64_t scalarArg;      // immediate scalar bits
  const void* scalarPtr;   // device scalar (ncclScalarDevice), read by the kernel
};


// One peer mapping of a registered allocation (refcounted per comm: a segment is imported once).
struct IpcMapping {
  int peer;
  uint64_t base;   // allocation base in the peer's address space
  IpcImport map;   // the same allocation as mapped here
  int refs;
};

// One registered allocation (reference struct ncclReg, src/include/register.h; src/register/register.cc): the
// whole allocation holding a registered buffer, mapped once into every peer's process (a peer's fd server
// imports it on request, ipc.cc) and refcounted by the ncclCommRegister handles (local) and the stream-capture
// auto-registrations (graph, NCCL_GRAPH_REGISTER) that lie in it.
struct RegAlloc {
  uint64_t base, size;
  uint64_t bufferId;   // the runtime's allocation id: a freed and re-allocated range is detected, never reused
  uint64_t tag;        // name of this registration at the peers' fd servers
  uint64_t rmt[NCCL_AMD_MAX_RANKS];  // the allocation's base as mapped in rank r's process (mine: base)
  bool imported[NCCL_AMD_MAX_RANKS]; // mapped by rank r's fd server (released by an RPC at deregistration)
  bool usable;         // every peer maps it: collectives on it may run zero-copy
  int localRefs, graphRefs;
  bool eagerRef;       // held by the eager registration cache (NCCL_AMD_EAGER_REGISTER=1, register.cc)
  uint64_t lastUse;    // the comm's registration clock at its last collective (eager cache eviction order)
  // recorded after every zero-copy kernel launched on it (outside captures): once complete, no kernel of this rank
  // hands the peers its addresses any more and no peer kernel reads it (each peer reads before its DONE signal,
  // which this rank's kernel waits for), so its peers' mappings may go without waiting for the device (regProgress)
  hipEvent_t lastEv;
  bool evMissing;      // lastEv could not be created: released only at a blocking entry point (after a device wait)
  int bouncePlans;     // a bounce allocation: planned collectives on it not launched yet (register.cc bounceFor)
};
enum RegRefKind { REF_LOCAL = 0, REF_GRAPH = 1, REF_EAGER = 2 };
// An eager collective whose buffers this rank could not register runs on the communicator's bounce allocation
// instead (register.cc bounceFor): its input copied in before the zero-copy kernel, its output copied out after.
struct BounceCopy {
  RegAlloc* ra;          // the bounce allocation's registration
  const void* userSend;  // nullptr: nothing to copy in (AllGather reads its own input in place)
  void* userRecv;
  char* send;            // in the bounce allocation (this process's address)
  char* recv;
  size_t sendBytes, recvBytes;
};
struct RegHandle {  // what ncclCommRegister returns
  void* buff;
  size_t size;
  RegAlloc* ra;  // nullptr when registration is disabled (NCCL_LOCAL_REGISTER=0)
};

enum CollFunc { FUNC_ALLREDUCE = 0, FUNC_REDUCESCATTER = 1, FUNC_ALLGATHER = 2, FUNC_REDUCE = 3, FUNC_COUNT = 4 };

// One collective's NCCL_ALGO / NCCL_PROTO enables (reference: the algoEnable / protoEnable rows of
// src/graph/tuning.cc:442-462), resolved onto this engine's kernels by loadTuning (enqueue.cc resolveFuncTuning).
struct FuncTuning {
  int algo;                 // TuneAlgoForce: exactly one implemented algorithm enabled forces it
  int oneShotOk, directOk;  // FORCE_NONE: which SIMPLE kernels the size table may pick
  int noAlgo;               // no enabled algorithm exists here: the collective fails (reference enqueue.cc:2052-2065)
  int llOn, simpleOn;       // protocols
  int ll128On;              // the LL64 line protocol (kernels.h): named in NCCL_PROTO, or NCCL_AMD_LL128=1
};

// Hot-path tuning knobs, read ONCE at communicator init (reference NCCL_PARAM caches its env reads,
// include/param.h:21-31) and agreed across ranks (rank 0's values win), so every rank takes the same
// algorithm/protocol decision and no getenv() runs per collective.
struct CommTuning {
  int checkPointers;        // NCCL_CHECK_POINTERS
  int forceElementwise;     // NCCL_AMD_FORCE_ELEMENTWISE (diagnostics)
  int protoFlags;           // NCCL_AMD_PROTO_FLAGS | (no release fence before data flags ? 8 : 0) | pulls
  int p2pFence;             // NCCL_AMD_P2P_FENCE: 1 fence, 0 none, -1 unset (none iff all ranks share one GPU)
  int linkChannels;         // channel budget of large plans at n >= 3 (enqueue.cc linkChannelBudget; 0 = none)
  FuncTuning fn[FUNC_COUNT];  // NCCL_ALGO / NCCL_PROTO per collective (reference grammar, enqueue.cc parseEnableList)
  int parseError;           // nonzero: NCCL_ALGO / NCCL_PROTO did not parse; every rank's init fails (ncclInvalidUsage)
  int symDisable;          // NCCL_AMD_SYM_DISABLE
  int symOneShot;           // NCCL_AMD_SYM_ONESHOT: caller promises out-of-place window AllReduces
  int symWtPublish;         // NCCL_AMD_SYM_WT: symmetric kernels publish with write-through stores, no L2 write-back
  int localRegister;        // NCCL_LOCAL_REGISTER: ncclCommRegister maps buffers into peers (zero-copy collectives)
  int graphRegister;        // NCCL_GRAPH_REGISTER: buffers of captured collectives are registered automatically
  int noAggregation;        // NCCL_AMD_NO_AGGREGATION
  int64_t oneShotBytes;     // NCCL_AMD_ONESHOT_BYTES
  int64_t llBytes;          // NCCL_AMD_LL_BYTES
  int64_t llChannelBytes;   // NCCL_AMD_LL_CHANNEL_BYTES
  int64_t ll128Bytes;       // NCCL_AMD_LL128_BYTES (upper end of the LL64 range)
  int64_t ll128ChannelBytes;  // NCCL_AMD_LL128_CHANNEL_BYTES
  int64_t minChannelBytes;  // NCCL_AMD_MIN_CHANNEL_BYTES
  int64_t oneShotChannelBytes;  // NCCL_AMD_ONESHOT_CHANNEL_BYTES
  int copyVariant;          // NCCL_AMD_COPY_VARIANT (nRanks == 1 copy kernel, diagnostics)
  int64_t copyGrid;         // NCCL_AMD_COPY_GRID (cap on its workgroups; default: one per 16 KiB tile)
  int64_t hostCopyGrid;     // NCCL_AMD_HOST_COPY_GRID (the cap when a buffer is pinned host memory; 0 = none)
  int copyXcdShift;         // NCCL_AMD_COPY_XCD_SHIFT (6): each XCD copies runs of 2^shift consecutive tiles
  int64_t ringChunkBytes;   // NCCL_ALGO=RING AllReduce chunk: NCCL_BUFFSIZE / NCCL_STEPS * ALLREDUCE_CHUNKSTEPS
  int refOrder;             // NCCL_AMD_REF_ORDER: AllReduce on the direct kernel in the reference's ring partition
  int refProto;             // ... of this protocol (NCCL_PROTO_LL 0, LL128 1, SIMPLE 2: the one NCCL_PROTO names)
  int64_t refChunkBytes;    // that protocol's ring chunk (NCCL_BUFFSIZE / NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE)
  int refChannels;          // NCCL_AMD_REF_NCHANNELS: the reference run's channel count K (0: the channel cap), <= 64
  int eagerRegister;        // NCCL_AMD_EAGER_REGISTER: unregistered buffers are registered on first use (register.cc)
  int64_t eagerBytes;       // NCCL_AMD_EAGER_REGISTER_BYTES: ... for collectives of at least this many bytes
  int eagerMax;             // NCCL_AMD_EAGER_REGISTER_MAX: eager registrations kept (LRU beyond it retired)
  int64_t eagerMaxBytes;    // NCCL_AMD_EAGER_REGISTER_MAX_BYTES: ... and their bytes
  // size table (NCCL_AMD_SIZE_TABLE, enqueue.cc sizeTable): per rank count, the upper ends of the LL, LL128-class
  // and one-shot ranges in bytes (0 = the built-in default); loaded once at init and agreed with rank 0's
  int64_t tableLL[NCCL_AMD_MAX_RANKS + 1], tableLL128[NCCL_AMD_MAX_RANKS + 1], tableOneShot[NCCL_AMD_MAX_RANKS + 1];
};
void loadTuning(CommTuning* t);  // enqueue.cc
// the size table's defaults for n ranks, then NCCL_AMD_SIZE_TABLE's rows over them (enqueue.cc; false: a bad file)
bool loadSizeTable(CommTuning* t, const char* path);
void resolveFence(CommTuning* t, bool oneDevice);  // enqueue.cc: the fence default, once devices are known
int linkChannelBudget(int nranks);                  // enqueue.cc: CU budget of large n >= 3 plans
int coResidentChannelCap(int minCUs, int ranksPerGpu);  // enqueue.cc: channels that stay co-resident per launch
void resolveLinkChannels(CommTuning* t, int nranks, bool userMaxCTAs);

struct ncclCommImpl;
}  // namespace ncclamd

// A registered window (reference struct ncclWindow_vidmem / ncclDevrWindow, src/dev_runtime.cc).
struct ncclWindow_vidmem {
  ncclComm* comm;
  void* userPtr;
  size_t size;
  int flags;
  char* peerPtr[NCCL_AMD_MAX_RANKS];  // every rank's window base as mapped in this process
  uint64_t peerBase[NCCL_AMD_MAX_RANKS];  // allocation bases of IPC-mapped peers (0: direct pointer)
};

// The opaque handle type of the public header.
struct ncclComm {
  uint64_t startMagic;
  int rank, nRanks, device;
  bool blocking;
  int minCTAs, maxCTAs;
  std::string commName;

  ncclamd::Bootstrap* bootstrap = nullptr;
  std::vector<ncclamd::PeerInfo> peers;

  // Device resources (transport.cc)
  void* staging = nullptr;          // local uncached staging area [ch][kind][slot][from][slotBytes]
  uint64_t* flags = nullptr;        // local uncached flag words [ch][flagKind][from]
  uint64_t* counters = nullptr;     // local connection step counters [ch][ctrKind][peer]
  void* peerStaging[NCCL_AMD_MAX_RANKS] = {};
  uint64_t* peerFlags[NCCL_AMD_MAX_RANKS] = {};
  ncclamd::IpcImport peerStagingMap[NCCL_AMD_MAX_RANKS] = {};  // other-process peers' slabs as mapped here
  ncclamd::IpcImport peerFlagsMap[NCCL_AMD_MAX_RANKS] = {};
  ncclamd::FdServer* fdServer = nullptr;  // serves this rank's exports to other processes (ipc.cc)
  ncclamd::DevComm* devComm = nullptr;  // device copy of the DevComm struct
  ncclamd::DevComm hostDevComm;          // host mirror
  uint32_t* hostAbort = nullptr;         // pinned, mapped: host→device abort flag
  uint32_t* hostError = nullptr;         // pinned, mapped: device→host error word
  size_t stagingAllocBytes = 0, flagsAllocBytes = 0, countersAllocBytes = 0;  // as allocated (ncclCommMemStats)
  size_t probeOffset = 0;  // mapping-check area in the flag allocation (mapcheck.cc), same on every rank
  size_t slotBytes = 0;
  int nSlots = 0;
  int maxChannels = 0;
  ncclamd::CommTuning tune;
  void* tunerCtx = nullptr;  // external tuner plugin context (tuner.cc)
  bool tunerLoaded = false;
  int llChannels = 32;      // LL protocol: channels and line bytes per (channel, parity, sender)
  size_t llBytes = 32 << 10;
  int chanCap = 0;  // channels per launch that stay co-resident even with several ranks per GPU
  // Several ranks of this process on this GPU (test mode): their spinning kernels must run concurrently,
  // but HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware queues, so two user streams
  // can share one queue and serialise the ranks (deadlock until the spin timeout). Such comms launch on
  // internalStream — created with a full CU mask, which always gets a hardware queue of its own — joined
  // to the user stream by evIn/evOut (graph capture follows the fork/join).
  bool sharedDevInProcess = false;
  hipStream_t internalStream = nullptr;
  hipEvent_t evIn = nullptr, evOut = nullptr;

  std::shared_ptr<ncclamd::LocalClique> clique;  // ncclCommInitAll comms: in-process all-gather
  std::vector<ncclWindow_vidmem*> windows;        // registered windows (register.cc)
  std::vector<ncclamd::IpcMapping> ipcMaps;
  std::vector<ncclamd::RegHandle*> regHandles;     // ncclCommRegister handles
  std::vector<ncclamd::RegAlloc*> regs;            // registered allocations (register.cc)
  // registrations no collective may use any more (stale, or their last graph reference gone inside a capture): their
  // peers' RELEASE requests go out at this rank's next blocking entry point, never inside a collective (register.cc)
  std::vector<ncclamd::RegAlloc*> regRetired;
  uint64_t regClock = 0;     // registration uses (RegAlloc::lastUse)
  ncclamd::RegAlloc* regLastUse[2] = {};  // the registrations regLookup's last hit returned (send, recv)
  size_t regScan = 0;        // regProgress: round-robin cursor of the freed-allocation check
  uint64_t regGen = 0;       // this comm's identity for graph-release tokens (0 until the first graph hold)
  bool warnedEagerCap = false;
  std::vector<std::pair<uint64_t, uint64_t>> eagerFailed;  // (base, buffer id) whose eager registration failed
  // the bounce allocation (register.cc bounceFor): registered with every peer once, grown on demand; grown-out ones
  // are freed at the next blocking entry point. bounceEv follows its last copy-out (uses on different streams wait).
  ncclamd::RegAlloc* bounce = nullptr;
  void* bounceMem = nullptr;
  hipEvent_t bounceEv = nullptr;
  std::vector<std::pair<ncclamd::RegAlloc*, void*>> bounceOld;
  bool bounceFailed = false;
  bool warnedEagerRefusal = false, warnedBounceMax = false;
  ncclamd::BounceCopy bounceNext = {};  // regLookup's last result when it bounced (bounceUsed)
  bool bounceUsed = false;

  std::vector<ncclamd::UserRedOp> userOps;
  std::atomic<int> asyncResult{ncclSuccess};
  bool finalized = false;
  bool destroyed = false;
  std::thread initThread;  // non-blocking ncclCommInitRankConfig (config.blocking = 0)
  uint64_t opCount = 0;
  uint32_t warnedAlgo = 0;  // NCCL_ALGO forced but unavailable for a collective: warned once per CollFunc
  bool warnedRefClamp = false;  // the reference-order channel count was clamped to MAXCHANNELS (warned once)
  // every rank can map every other-process peer's registered buffers (each such peer runs an fd server): derived
  // from the shared peer table at init, so every rank takes the same registered / staged decision (register.cc)
  bool regIpcAll = false;
  bool multiProcess = false;  // some peer lives in another process (shared peer table: the same on every rank)
  uint64_t endMagic;
};

namespace ncclamd {

ncclResult_t commCheck(const ncclComm* comm, const char* opname, const char* what);
// a device-side error recorded by a kernel (timeout, abort, kernel mismatch) becomes the comm's async error (init.cc)
void commPollAsync(ncclComm* comm);
ncclResult_t transportSetup(ncclComm* comm);     // allocate staging/flags + IPC export
ncclResult_t transportConnect(ncclComm* comm);   // map peers after the PeerInfo exchange
ncclResult_t transportFree(ncclComm* comm);
ncclResult_t transportDrainCredits(ncclComm* comm);  // wait for acks peers still owe (destroy)
ncclResult_t commAllocDevState(ncclComm* comm);  // counters, DevComm upload, abort/error words
size_t commDeviceBytes(const ncclComm* comm);     // device memory held (ncclCommMemStats)

// ---------------------------------------------------------------- mapping check (mapcheck.cc)
// At init, every rank writes a pattern into every peer's staging slab and flag block THROUGH its mapping of them and
// reads back the peers' own patterns the same way; a mapping that does not carry the bytes fails the init with
// ncclSystemError naming the device pair, the allocation, the direction and the import path.
constexpr size_t kMapProbeBytes = 2 * NCCL_AMD_MAX_RANKS * 16;
uint64_t mapCheckWord(uint64_t nonce, int kind, int src, int dst, int half);  // expected word (kind: 0 staging, 1 flags)
struct MapCheckObs {
  // got[kind][peer][half]: written by `peer` into MY allocation (dir 0), read by me from peer's (dir 1)
  uint64_t wrote[2][NCCL_AMD_MAX_RANKS][2];
  uint64_t read[2][NCCL_AMD_MAX_RANKS][2];
};
struct MapCheckPeer {  // how this rank reaches peer r (for the message)
  int device;
  char busId[32];
  const char* path;    // how this rank maps r's memory: same-GPU pointer, peer pointer, dma-buf import, hipIpc handle
  const char* pathIn;  // how r maps this rank's memory (as far as this rank knows: what it exported)
};
// The failures of one rank's observations, one line each ("" = every mapping carried the patterns).
std::string mapCheckVerify(int me, int nRanks, uint64_t nonce, const MapCheckObs& obs, const MapCheckPeer* peers);
ncclResult_t mapCheck(const std::vector<ncclComm*>& comms);  // the check for these local comms (init.cc)
// Re-import peer r's staging slab and flag block through the hipIpc handles of their exports (the dma-buf import's
// fallback) and refresh the device's view of them; ncclSystemError when peer r has no such handle (transport.cc).
ncclResult_t transportRemapPeer(ncclComm* comm, int r);
ncclResult_t launchMapCheck(const DevComm* dc, const MapCheckArgs& a, uint64_t* out, hipStream_t stream);  // kernels.hip

// ---------------------------------------------------------------- enqueue (reference src/enqueue.cc)
struct CollInfo {  // reference: struct ncclInfo, src/include/info.h:17-41
  CollFunc func;
  const char* opName;
  const void* sendbuff;
  void* recvbuff;
  size_t count;
  ncclDataType_t datatype;
  ncclRedOp_t op;
  int root;
  ncclComm* comm;
  hipStream_t stream;
};

enum Algo { ALGO_COPY = 0, ALGO_ONERANK = 1, ALGO_DIRECT = 2, ALGO_ONESHOT = 3, ALGO_LL = 4, ALGO_PIPE = 5 };
// NCCL_ALGO values of CommTuning::algo
enum TuneAlgoForce { FORCE_NONE = 0, FORCE_ONESHOT = 1, FORCE_DIRECT = 2, FORCE_RING = 3, FORCE_TREE = 4 };

struct LaunchPlan {  // one kernel launch (reference: struct ncclKernelPlan, src/include/comm.h)
  CollFunc func;
  int algo;
  ncclDataType_t datatype;
  int eltSize;
  int devOp;
  int nChannels;
  size_t bytes;
  hipStream_t stream;
  CollArgs args;
  LLBatchArgs ll;  // ALGO_LL
  CollBatchArgs batch;  // ALGO_DIRECT / ALGO_ONESHOT group batch when batch.nOps > 1 (collBatchKernel)
  int copyVariant;  // ALGO_COPY
  int64_t copyGrid;
  int copyXcdShift;
  int pipeKind;     // ALGO_PIPE: PipeKind (pipe.h)
};

ncclResult_t enqueueCheck(CollInfo* info);
// plan + launch (enqueue.cc); forkJoin=false: the caller (group end) forks/joins shared-GPU comms itself
ncclResult_t launchColl(const CollInfo& info, bool forkJoin = true);
ncclResult_t collFork(const CollInfo& info);
void collProgress(ncclComm* comm, hipStream_t stream);  // enqueue.cc: registration / release upkeep on the collective path, never waiting
bool llPlan(const CollInfo& info, LLOp* op);                  // LL eligibility + plan (enqueue.cc)

// ---------------------------------------------------------------- tuner plugin (reference src/plugin/tuner.cc)
enum TuneAlgo { TUNE_DEFAULT = 0, TUNE_LL = 1, TUNE_ONESHOT = 2, TUNE_DIRECT = 3, TUNE_LL128 = 4 };
ncclResult_t tunerLoad(ncclComm* comm);
void tunerUnload(ncclComm* comm);
void tunerPick(ncclComm* comm, CollFunc func, size_t bytes, int numPipeOps, int llMask, int regBuff, int* algo, int* nch);
// the engine's cost model (tuner.cc): µs of fixed latency + µs of the busiest resource's transfer time
enum ModelAlgo { MODEL_COPY, MODEL_LL, MODEL_LL128, MODEL_ONESHOT, MODEL_DIRECT, MODEL_SYM, MODEL_RING, MODEL_CHAIN };
struct ModelCost {
  double latUs, xferUs;
  double total() const { return latUs + xferUs; }
};
ModelCost modelCost(ModelAlgo a, CollFunc func, int n, size_t bytes);
ncclResult_t collJoin(const CollInfo& info);
ncclResult_t launchPlan(const LaunchPlan& plan);  // kernels.hip

struct SymPlan {  // one symmetric (window) kernel launch
  int coll;       // SymColl (kernels.h)
  ncclDataType_t datatype;
  int eltSize;
  int devOp;
  int nChannels;
  hipStream_t stream;
  SymArgs args;
  RegAlloc* regUse[2];  // registered mode: the send / recv registrations it runs on (their lastEv, register.cc)
  bool bounced;         // runs on the bounce allocation: `bounce` copies around the launch (bounceLaunch)
  BounceCopy bounce;
};
ncclResult_t launchSymPlan(const SymPlan& plan);  // kernels.hip

// planColl's outcome: a kernel launch (LaunchPlan), a symmetric-window launch (SymPlan) or nothing
enum PlanKind { PLAN_KERNEL = 0, PLAN_SYM = 1, PLAN_NONE = 2 };
struct PlannedColl {  // one op of a group, planned (group.cc)
  CollInfo info;
  int kind;
  LaunchPlan p;
  SymPlan sp;
};
ncclResult_t planColl(const CollInfo& info, LaunchPlan& p, SymPlan& sp, int* kind);
bool batchable(const std::vector<PlannedColl>& run, const PlannedColl& b);  // can b join run's launch?
ncclResult_t launchBatch(std::vector<PlannedColl>& run);  // one launch for a run of batchable ops
// window lookup: the window holding [p, p+bytes) with NCCL_WIN_COLL_SYMMETRIC, or nullptr (register.cc)
ncclWindow_vidmem* findSymWindow(ncclComm* comm, const void* p, size_t bytes);
// Registered buffers of one collective (register.cc): true when [send, +sendBytes) (skipped when send is
// nullptr) and [recv, +recvBytes) lie in allocations every peer maps — registered with ncclCommRegister, or,
// under stream capture with NCCL_GRAPH_REGISTER=1, registered here on the fly. rmtSend[r] / rmtRecv[r] = the
// buffers as mapped in rank r's process (mine: the buffers themselves).
// With `eager` (NCCL_AMD_EAGER_REGISTER=1 and an eligible op), unregistered allocations are registered here too.
bool regLookup(ncclComm* comm, hipStream_t stream, const void* send, size_t sendBytes, const void* recv,
               size_t recvBytes, const char** rmtSend, char** rmtRecv, bool eager = false);
// release every window and IPC mapping (destroy: also asks peers to unmap this rank's registrations; abort: not)
void windowsFree(ncclComm* comm, bool notifyPeers);
// at init: one plain allocation per rank registered with and read back by every peer; any failure turns the eager
// zero-copy default off on every rank (register.cc)
ncclResult_t eagerProbe(ncclComm* comm);
// A blocking entry point's registration upkeep (register.cc): graph-held references whose graphs are gone are
// dropped, stale and surplus eager registrations released, and retired registrations' RELEASE requests sent.
void regBlockingPoint(ncclComm* comm);
// The same upkeep on the collective path, never waiting (register.cc): freed allocations found, the eager cache kept
// within its count and byte bounds, and RELEASE sent for retired registrations whose last kernel completed.
void regProgress(ncclComm* comm);
// after a launched zero-copy plan: its registrations' lastEv recorded on its stream (outside captures)
void regRecordUse(ncclComm* comm, const SymPlan& sp);
// a zero-copy plan on the bounce allocation (sp.bounced): launched between its copy-in and copy-out (register.cc)
ncclResult_t bounceLaunch(ncclComm* comm, const SymPlan& sp);
// Set by ncclGroupSimulateEnd around its planning (group.cc): an eager lookup then registers nothing and reports the
// zero-copy plan the real group end would take (register.cc regLookup).
extern thread_local bool tPlanOnly;
// [p, +bytes) lies in a usable registration held by an ncclCommRegister handle (no side effects)
bool regCovers(ncclComm* comm, const void* p, size_t bytes);
// all-gather over the comm's bootstrap (multi-process) or in-process clique (ncclCommInitAll)
ncclResult_t commAllGather(ncclComm* comm, void* data, size_t bytesPerRank);
ncclResult_t launchCopy(void* dst, const void* src, size_t bytes, hipStream_t stream, int variant, int64_t gridCap,
                        int xcdShift);
ncclResult_t warmKernels();  // load all kernel code objects on the current device (kernels.hip)
int typeSize(ncclDataType_t t);

// ---------------------------------------------------------------- groups (reference src/group.cc)
ncclResult_t groupStartInternal();
ncclResult_t groupEndInternal(ncclSimInfo_t* simInfo = nullptr);  // simInfo: ncclGroupSimulateEnd
bool groupActive();
void groupRecordError(ncclResult_t r);
ncclResult_t groupDeferColl(const CollInfo& info);
ncclResult_t groupDeferInit(std::function<ncclResult_t()> job);

// Restores the caller's current device when an API call that switched to its comm's device returns (the
// reference saves and restores around every launch and registration: enqueue.cc:3137-3162, group.cc:860-863).
struct DeviceRestore {
  int dev = -1;
  DeviceRestore() { (void)hipGetDevice(&dev); }
  ~DeviceRestore() {
    int cur = -1;
    if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
  }
};

}  // namespace ncclamd
