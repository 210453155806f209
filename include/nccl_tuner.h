/*
 * nccl_tuner.h — tuner plugin ABI understood by the MI355X engine (libnccl.so).
 *
 * Same layouts and symbol names as the reference's tuner plugin interface, versions 4-6
 * (/root/reference/src/include/plugin/tuner/tuner_v4.h, tuner_v5.h, tuner_v6.h:12-83;
 * plugins/tuner/basic/nccl/{common,tuner}.h for the enums), so an existing NCCL tuner plugin
 * (`ncclTunerPlugin_v6` / `_v5` / `_v4` exported from `libnccl-tuner-<name>.so`, selected with
 * NCCL_TUNER_PLUGIN) loads unchanged. How the engine maps the cost table onto its own algorithms is
 * in DESIGN.md §10.4.
 */
#ifndef NCCL_TUNER_H_
#define NCCL_TUNER_H_

#include <stddef.h>
#include <stdint.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* plugins/tuner/basic/nccl/common.h:11-14 */
typedef enum {
  NCCL_LOG_NONE = 0, NCCL_LOG_VERSION = 1, NCCL_LOG_WARN = 2, NCCL_LOG_INFO = 3, NCCL_LOG_ABORT = 4, NCCL_LOG_TRACE = 5
} ncclDebugLogLevel;
typedef void (*ncclDebugLogger_t)(ncclDebugLogLevel level, unsigned long flags, const char* file, int line,
                                  const char* fmt, ...);

/* plugins/tuner/basic/nccl/tuner.h:17-46 */
typedef enum {
  ncclFuncBroadcast = 0, ncclFuncReduce = 1, ncclFuncAllGather = 2, ncclFuncReduceScatter = 3,
  ncclFuncAllReduce = 4, ncclFuncSendRecv = 5, ncclFuncSend = 6, ncclFuncRecv = 7, ncclNumFuncs = 8
} ncclFunc_t;

#define NCCL_NUM_ALGORITHMS 7
#define NCCL_ALGO_UNDEF -1
#define NCCL_ALGO_TREE 0
#define NCCL_ALGO_RING 1
#define NCCL_ALGO_COLLNET_DIRECT 2
#define NCCL_ALGO_COLLNET_CHAIN 3
#define NCCL_ALGO_NVLS 4
#define NCCL_ALGO_NVLS_TREE 5
#define NCCL_ALGO_PAT 6

#define NCCL_NUM_PROTOCOLS 3
#define NCCL_PROTO_UNDEF -1
#define NCCL_PROTO_LL 0
#define NCCL_PROTO_LL128 1
#define NCCL_PROTO_SIMPLE 2

#define NCCL_ALGO_PROTO_IGNORE -1.0

/* tuner_v5.h: NVLink-domain info and tuning constants (passed to init; this engine fills what
 * applies to one xGMI node and leaves the rest zero) */
typedef struct {
  int nNvlDomains;
  int minRanksPerNvlDomain;
  int maxRanksPerNvlDomain;
} ncclNvlDomainInfo_v5_t;

#define NCCL_NUM_HW_LINKS_V5 3
#define NCCL_NUM_COMPCAPS_V5 4
#define NCCL_NUM_TUNING_SCALES_V5 3
typedef struct {
  double baseLatencies[NCCL_NUM_ALGORITHMS][NCCL_NUM_PROTOCOLS];
  double hwLatencies[NCCL_NUM_HW_LINKS_V5][NCCL_NUM_ALGORITHMS][NCCL_NUM_PROTOCOLS];
  double llMaxBws[NCCL_NUM_COMPCAPS_V5][NCCL_NUM_TUNING_SCALES_V5];
  double perChMaxRingLL128Bws[NCCL_NUM_COMPCAPS_V5][NCCL_NUM_TUNING_SCALES_V5];
  double perChMaxTreeLL128Bws[NCCL_NUM_COMPCAPS_V5][NCCL_NUM_TUNING_SCALES_V5];
  double perChMaxTreeBws[NCCL_NUM_COMPCAPS_V5][NCCL_NUM_TUNING_SCALES_V5];
  double perChMaxNVLSTreeBws[NCCL_NUM_COMPCAPS_V5][NCCL_NUM_TUNING_SCALES_V5];
} ncclTunerConstants_v5_t;
typedef ncclNvlDomainInfo_v5_t ncclNvlDomainInfo_v6_t;
typedef ncclTunerConstants_v5_t ncclTunerConstants_v6_t;

/* tuner_v6.h:19-83 */
typedef struct {
  const char* name;
  ncclResult_t (*init)(void** ctx, uint64_t commId, size_t nRanks, size_t nNodes, ncclDebugLogger_t logFunction,
                       ncclNvlDomainInfo_v6_t* nvlDomainInfo, ncclTunerConstants_v6_t* constants);
  ncclResult_t (*getCollInfo)(void* context, ncclFunc_t collType, size_t nBytes, int numPipeOps,
                              float** collCostTable, int numAlgo, int numProto, int regBuff, int* nChannels);
  ncclResult_t (*finalize)(void* context);
  ncclResult_t (*getChunkSize)(void* context, ncclFunc_t collType, size_t nBytes, int algo, int proto,
                               int nChannels, size_t* chunkSize);
} ncclTuner_v6_t;

/* tuner_v5.h */
typedef struct {
  const char* name;
  ncclResult_t (*init)(void** ctx, uint64_t commId, size_t nRanks, size_t nNodes, ncclDebugLogger_t logFunction,
                       ncclNvlDomainInfo_v5_t* nvlDomainInfo, ncclTunerConstants_v5_t* constants);
  ncclResult_t (*getCollInfo)(void* context, ncclFunc_t collType, size_t nBytes, int numPipeOps,
                              float** collCostTable, int numAlgo, int numProto, int regBuff, int* nChannels);
  ncclResult_t (*finalize)(void* context);
} ncclTuner_v5_t;

/* tuner_v4.h */
typedef struct {
  const char* name;
  ncclResult_t (*init)(size_t nRanks, size_t nNodes, ncclDebugLogger_t logFunction, void** context);
  ncclResult_t (*getCollInfo)(void* context, ncclFunc_t collType, size_t nBytes, int numPipeOps,
                              float** collCostTable, int numAlgo, int numProto, int regBuff, int* nChannels);
  ncclResult_t (*destroy)(void* context);
} ncclTuner_v4_t;

#ifdef __cplusplus
}
#endif

#endif /* NCCL_TUNER_H_ */
