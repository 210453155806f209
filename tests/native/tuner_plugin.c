/* tuner_plugin.c — a test tuner plugin built against include/nccl_tuner.h (the reference's ABI v6),
 * loaded by libnccl.so through NCCL_TUNER_PLUGIN. Behaviour from the environment:
 *   TEST_TUNER_FORCE = ring_simple | tree_simple | ring_ll | none (leave the table alone)
 *   TEST_TUNER_NCH   = channel count to request (0: none)
 * testTunerCalls() reports how many getCollInfo calls were made, testTunerLastFunc() the last collType. */
#include <stdlib.h>
#include <string.h>

#include "nccl_tuner.h"

static int gCalls = 0;
static int gLastFunc = -1;
static int gInits = 0;

__attribute__((visibility("default"))) int testTunerCalls(void) { return gCalls; }
__attribute__((visibility("default"))) int testTunerLastFunc(void) { return gLastFunc; }
__attribute__((visibility("default"))) int testTunerInits(void) { return gInits; }

static ncclResult_t pInit(void** ctx, uint64_t commId, size_t nRanks, size_t nNodes, ncclDebugLogger_t log,
                          ncclNvlDomainInfo_v6_t* dom, ncclTunerConstants_v6_t* consts) {
  (void)commId; (void)nNodes; (void)dom; (void)consts;
  if (log) log(NCCL_LOG_INFO, 0, __FILE__, __LINE__, "test tuner init for %zu ranks", nRanks);
  *ctx = malloc(16);
  gInits++;
  return ncclSuccess;
}

static ncclResult_t pGetCollInfo(void* ctx, ncclFunc_t collType, size_t nBytes, int numPipeOps, float** costTable,
                                 int numAlgo, int numProto, int regBuff, int* nChannels) {
  (void)ctx; (void)nBytes; (void)numPipeOps; (void)regBuff;
  float (*table)[NCCL_NUM_PROTOCOLS] = (float (*)[NCCL_NUM_PROTOCOLS])costTable;
  gCalls++;
  gLastFunc = (int)collType;
  const char* force = getenv("TEST_TUNER_FORCE");
  int a = -1, p = -1;
  if (force && !strcmp(force, "ring_simple")) a = NCCL_ALGO_RING, p = NCCL_PROTO_SIMPLE;
  if (force && !strcmp(force, "tree_simple")) a = NCCL_ALGO_TREE, p = NCCL_PROTO_SIMPLE;
  if (force && !strcmp(force, "ring_ll")) a = NCCL_ALGO_RING, p = NCCL_PROTO_LL;
  if (a >= 0 && a < numAlgo && p < numProto && table[a][p] != NCCL_ALGO_PROTO_IGNORE) table[a][p] = 0.0f;
  const char* nch = getenv("TEST_TUNER_NCH");
  if (nch) *nChannels = atoi(nch);
  return ncclSuccess;
}

static ncclResult_t pFinalize(void* ctx) {
  free(ctx);
  return ncclSuccess;
}

__attribute__((visibility("default"))) const ncclTuner_v6_t ncclTunerPlugin_v6 = {
    "mi355x-test", pInit, pGetCollInfo, pFinalize, NULL};
