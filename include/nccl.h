/*
 * nccl.h — C ABI of the MI355X tensor-bucket reduction engine (libnccl.so, nccl_amd).
 *
 * This header re-declares the subset of the NCCL 2.30.7 public API that the device-resident
 * reduction path needs, with the SAME enum values, struct layouts and function signatures as the
 * reference header template /root/reference/src/nccl.h.in, so that existing NCCL callers compile
 * and link against this library unchanged. The only type difference is the stream: the reference's
 * cudaStream_t (nccl.h.in:455-532) is hipStream_t here — both are pointer-sized opaque handles, so
 * the calling convention is identical.
 *
 * Each declaration cites the reference declaration it replaces (nccl.h.in:<line>).
 * Every function is also exported under a `pnccl` profiling alias (reference: src/include/core.h:16-27,
 * src/libnccl.map:13-19).
 */
#ifndef NCCL_H_
#define NCCL_H_

#include <hip/hip_runtime_api.h>
#include <limits.h>
#include <stdint.h>
#include <stddef.h>

/* Version: the reference snapshot is 2.30.7 (makefiles/version.mk:9-11); NCCL_VERSION() is the
 * encoding of nccl.h.in:26. */
#define NCCL_MAJOR 2
#define NCCL_MINOR 30
#define NCCL_PATCH 7
#define NCCL_SUFFIX "-mi355x"
#define NCCL_VERSION(X, Y, Z) (((X) <= 2 && (Y) <= 8) ? (X) * 1000 + (Y) * 100 + (Z) : (X) * 10000 + (Y) * 100 + (Z))
#define NCCL_VERSION_CODE NCCL_VERSION(NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH)

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque communicator handle (nccl.h.in:35). */
typedef struct ncclComm* ncclComm_t;
#define NCCL_COMM_NULL NULL

/* Opaque registered-memory window (nccl.h.in:37). */
typedef struct ncclWindow_vidmem* ncclWindow_t;

/* Window flags (nccl.h.in:64-68). NCCL_WIN_COLL_SYMMETRIC: every rank registers a buffer of the same size
 * and passes buffers at the same offset inside it to collectives, which may then read and write peers'
 * windows directly (zero-copy symmetric kernels). */
#define NCCL_WIN_DEFAULT 0x00
#define NCCL_WIN_COLL_SYMMETRIC 0x01
#define NCCL_WIN_STRICT_ORDERING 0x02
#define NCCL_WIN_REQUIRED_ALIGNMENT 4096

/* 128-byte opaque rendezvous id (nccl.h.in:40-41). */
#define NCCL_UNIQUE_ID_BYTES 128
typedef struct {
  char internal[NCCL_UNIQUE_ID_BYTES];
} ncclUniqueId;

/* Result codes (nccl.h.in:44-53). Values are ABI. */
typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1, /* a HIP runtime call failed */
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclTimeout = 8,
  ncclNumResults = 9
} ncclResult_t;

#define NCCL_CONFIG_UNDEF_INT INT_MIN
#define NCCL_CONFIG_UNDEF_PTR NULL
#define NCCL_SPLIT_NOCOLOR -1
#define NCCL_UNDEF_FLOAT -1.0f
#define NCCL_API_MAGIC 0xcafebeef

#define NCCL_CTA_POLICY_DEFAULT 0x00
#define NCCL_CTA_POLICY_EFFICIENCY 0x01
#define NCCL_CTA_POLICY_ZERO 0x02

/* Communicator configuration (nccl.h.in:84-108): identical field order and types, so a
 * ncclConfig_t built by a caller against the reference header is read correctly here.
 * Fields honoured by this engine: blocking, minCTAs, maxCTAs, commName. The rest are accepted
 * and ignored (their subsystems — CGA clusters, net, collnet, NVLS, RMA — do not exist on the
 * MI355X intra-node path). */
typedef struct ncclConfig_v23000 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
  int trafficClass;
  const char* commName;
  int collnetEnable;
  int CTAPolicy;
  int shrinkShare;
  int nvlsCTAs;
  int nChannelsPerNetPeer;
  int nvlinkCentricSched;
  int graphUsageMode;
  int numRmaCtx;
  int maxP2pPeers;
  int graphStreamOrdering;
} ncclConfig_t;

/* nccl.h.in:112-134 */
#define NCCL_CONFIG_INITIALIZER                                                                      \
  {                                                                                                  \
    sizeof(ncclConfig_t), NCCL_API_MAGIC, NCCL_VERSION_CODE, NCCL_CONFIG_UNDEF_INT,                  \
        NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_PTR,  \
        NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_PTR, NCCL_CONFIG_UNDEF_INT,  \
        NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,  \
        NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,  \
        NCCL_CONFIG_UNDEF_INT                                                                        \
  }

/* Reduction operators (nccl.h.in:363-379). Values are ABI. */
typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;
typedef enum {
  ncclSum = 0,
  ncclProd = 1,
  ncclMax = 2,
  ncclMin = 3,
  ncclAvg = 4,
  ncclNumOps = 5,
  ncclMaxRedOp = 0x7fffffff >> (32 - 8 * sizeof(ncclRedOp_dummy_t))
} ncclRedOp_t;

/* Element types (nccl.h.in:382-395). Values are ABI. */
typedef enum {
  ncclInt8 = 0, ncclChar = 0,
  ncclUint8 = 1,
  ncclInt32 = 2, ncclInt = 2,
  ncclUint32 = 3,
  ncclInt64 = 4,
  ncclUint64 = 5,
  ncclFloat16 = 6, ncclHalf = 6,
  ncclFloat32 = 7, ncclFloat = 7,
  ncclFloat64 = 8, ncclDouble = 8,
  ncclBfloat16 = 9,
  ncclFloat8e4m3 = 10,
  ncclFloat8e5m2 = 11,
  ncclNumTypes = 12
} ncclDataType_t;

/* Scalar residence for ncclRedOpCreatePreMulSum (nccl.h.in:398-407). */
typedef enum { ncclScalarDevice = 0, ncclScalarHostImmediate = 1 } ncclScalarResidence_t;

/* ---- Library / communicator lifecycle ---- */

/* nccl.h.in:156,159 — device allocation helpers (plain hipMalloc-backed here). */
ncclResult_t ncclMemAlloc(void** ptr, size_t size);
ncclResult_t pncclMemAlloc(void** ptr, size_t size);
ncclResult_t ncclMemFree(void* ptr);
ncclResult_t pncclMemFree(void* ptr);

/* nccl.h.in:166 */
ncclResult_t ncclGetVersion(int* version);
ncclResult_t pncclGetVersion(int* version);

/* nccl.h.in:172 — rendezvous id for ncclCommInitRank (TCP bootstrap root address + magic). */
ncclResult_t ncclGetUniqueId(ncclUniqueId* uniqueId);
ncclResult_t pncclGetUniqueId(ncclUniqueId* uniqueId);

/* nccl.h.in:177 */
ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank,
                                    ncclConfig_t* config);
ncclResult_t pncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank,
                                     ncclConfig_t* config);

/* nccl.h.in:186 — one rank per process or thread; the current HIP device is the rank's device. */
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);
ncclResult_t pncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);

/* nccl.h.in:263 — several ids (same number and order on every rank); this single-node star rendezvouses at
 * commIds[0] and tells the other ids' roots to exit. */
ncclResult_t ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
                                      ncclUniqueId* commIds, ncclConfig_t* config);
ncclResult_t pncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
                                       ncclUniqueId* commIds, ncclConfig_t* config);

/* nccl.h.in:195 — single-process clique, one comm per device in devlist (NULL = 0..ndev-1). */
ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);
ncclResult_t pncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);

/* nccl.h.in:203,207,212 */
ncclResult_t ncclCommFinalize(ncclComm_t comm);
ncclResult_t pncclCommFinalize(ncclComm_t comm);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t pncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclCommAbort(ncclComm_t comm);
ncclResult_t pncclCommAbort(ncclComm_t comm);

/* nccl.h.in:267,271 */
const char* ncclGetErrorString(ncclResult_t result);
const char* pncclGetErrorString(ncclResult_t result);
const char* ncclGetLastError(ncclComm_t comm);
const char* pncclGetLastError(ncclComm_t comm);

/* nccl.h.in:286,290,294,298 */
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
ncclResult_t pncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
ncclResult_t ncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t pncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t pncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank);
ncclResult_t pncclCommUserRank(const ncclComm_t comm, int* rank);

/* nccl.h.in:333-348 — device memory the communicator holds (all of it persistent: nothing is suspendable). */
typedef enum {
  ncclStatGpuMemSuspend = 0,
  ncclStatGpuMemSuspended = 1,
  ncclStatGpuMemPersist = 2,
  ncclStatGpuMemTotal = 3
} ncclCommMemStat_t;
ncclResult_t ncclCommMemStats(ncclComm_t comm, ncclCommMemStat_t stat, uint64_t* value);
ncclResult_t pncclCommMemStats(ncclComm_t comm, ncclCommMemStat_t stat, uint64_t* value);

/* ---- Buffer registration (nccl.h.in:301-307, 350-360) ---- */
/* nccl.h.in:302 — local (non-collective) registration hint; see DESIGN.md §10.3. */
ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
ncclResult_t pncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
/* nccl.h.in:306 */
ncclResult_t ncclCommDeregister(const ncclComm_t comm, void* handle);
ncclResult_t pncclCommDeregister(const ncclComm_t comm, void* handle);
/* nccl.h.in:351 — collective over the communicator (inside a group when one thread drives several ranks). */
ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win, int winFlags);
ncclResult_t pncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win, int winFlags);
/* nccl.h.in:355 */
ncclResult_t ncclCommWindowDeregister(ncclComm_t comm, ncclWindow_t win);
ncclResult_t pncclCommWindowDeregister(ncclComm_t comm, ncclWindow_t win);
/* nccl.h.in:359 */
ncclResult_t ncclWinGetUserPtr(ncclComm_t comm, ncclWindow_t win, void** outUserPtr);
ncclResult_t pncclWinGetUserPtr(ncclComm_t comm, ncclWindow_t win, void** outUserPtr);

/* ---- Custom reduction operators (nccl.h.in:418-431) ---- */
ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                      ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t pncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                       ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);
ncclResult_t pncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);

/* ---- Collectives: asynchronous, enqueued on `stream` (nccl.h.in:433-442) ---- */

/* nccl.h.in:455 — result at `root` only; recvbuff may be NULL elsewhere. In-place iff send==recv. */
ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                        ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                         ncclRedOp_t op, int root, ncclComm_t comm, hipStream_t stream);

/* nccl.h.in:496 — in-place iff sendbuff == recvbuff. */
ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                            ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);

/* nccl.h.in:512 — sendbuff holds nranks*recvcount elements; in-place iff
 * recvbuff == sendbuff + rank*recvcount. */
ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                               ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                                ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);

/* nccl.h.in:529 — recvbuff holds nranks*sendcount elements; in-place iff
 * sendbuff == recvbuff + rank*sendcount. */
ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream);
ncclResult_t pncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                            ncclComm_t comm, hipStream_t stream);

/* ---- Group semantics (nccl.h.in:700-735) ---- */
ncclResult_t ncclGroupStart(void);
ncclResult_t pncclGroupStart(void);
ncclResult_t ncclGroupEnd(void);
ncclResult_t pncclGroupEnd(void);

/* nccl.h.in:136-152, 741 — plan the group's collectives without launching them and return the cost model's
 * estimate (microseconds, like the reference's tuning table) in simInfo->estimatedTime. */
typedef struct ncclSimInfo_v22200 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  float estimatedTime;
} ncclSimInfo_t;
#define NCCL_SIM_INFO_INITIALIZER \
  { sizeof(ncclSimInfo_t), 0x74685283, NCCL_VERSION_CODE, NCCL_UNDEF_FLOAT }
ncclResult_t ncclGroupSimulateEnd(ncclSimInfo_t* simInfo);
ncclResult_t pncclGroupSimulateEnd(ncclSimInfo_t* simInfo);

#ifdef __cplusplus
}
#endif

#endif /* NCCL_H_ */
