// plan_test.cc — CPU test driver for the host-side planning of enqueue.cc (size table, protocol and
// algorithm choice, channel/slice plan, NCCL_ALGO / NCCL_PROTO handling). It is compiled together with
// enqueue.cc and debug.cc (no GPU, no HIP runtime): the launch entry points and the few HIP runtime calls
// enqueue.cc makes are stubbed so every plan is recorded and printed instead of launched.
//
//   plan_test NRANKS FUNC(ar|rs|ag|reduce) DTYPE COUNT [ALIGN_OFFSET_BYTES] [CHANCAP]
// prints one line: algo=<copy|onerank|direct|oneshot|ll|ring|chain> nch=<channels> part=<elements|payloads>
//                  slice=<elements> steps=<n> chunk=<elements> (ring / chain also: kind= cbdlo= cbdhi=)
//   plan_test NRANKS batch FUNC:DTYPE:COUNT[:OP] ...
// plans the ops as one group (enqueue.cc planColl / batchable / launchBatch, in group.cc's order) and prints one
// line per launch: algo=<...> ops=<ops in the launch> grid=<workgroups> ranges=<chOff+nch per op, comma-separated>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../nccl_amd/csrc/core.h"

// ---- HIP runtime stubs (enqueue.cc only sets the device, queries attributes and records events) ----
extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub"; }
hipError_t hipPointerGetAttributes(hipPointerAttribute_t*, const void*) { return hipErrorInvalidValue; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* st) {
  *st = hipStreamCaptureStatusNone;
  return hipSuccess;
}
}

namespace ncclamd {
static LaunchPlan gPlan;
static SymPlan gSym;
static int gKind = -1;  // 0 LaunchPlan, 1 SymPlan
static bool gBatchMode = false;
static const char* kAlgoNames[] = {"copy", "onerank", "direct", "oneshot", "ll", "pipe"};
ncclResult_t launchPlan(const LaunchPlan& p) {
  gPlan = p;
  gKind = 0;
  if (gBatchMode) {  // one line per launch
    printf("algo=%s", kAlgoNames[p.algo]);
    if (p.algo == ALGO_LL) {
      printf(" ops=%d grid=%d ranges=", p.ll.nOps, p.nChannels);
      for (int k = 0; k < p.ll.nOps; k++) printf("%s%d+%d", k ? "," : "", p.ll.ops[k].chOff, p.ll.ops[k].nch);
      if (p.ll.nOps > 1) {  // per channel: the ops it runs (LLArgs::chMask)
        printf(" masks=");
        for (int c = 0; c < kMaxLLChannels; c++) printf("%s%x", c ? "," : "", p.ll.chMask[c]);
      }
    } else if (p.batch.nOps > 1) {
      printf(" ops=%d grid=%d ranges=", p.batch.nOps, p.nChannels);
      for (int k = 0; k < p.batch.nOps; k++) printf("%s%d+%d", k ? "," : "", p.batch.chOff[k], p.batch.nch[k]);
    } else {
      printf(" ops=1 grid=%d ranges=0+%d", p.nChannels, p.nChannels);
    }
    printf("\n");
  }
  return ncclSuccess;
}
ncclResult_t launchSymPlan(const SymPlan& p) {
  gSym = p;
  gKind = 1;
  return ncclSuccess;
}
ncclWindow_vidmem* findSymWindow(ncclComm*, const void*, size_t) { return nullptr; }
// eager registration (NCCL_AMD_EAGER_REGISTER=1) of an eligible op succeeds: the plan shows the zero-copy kernel
bool regLookup(ncclComm*, hipStream_t, const void*, size_t, const void*, size_t, const char**, char**, bool eager) {
  return eager;
}
bool groupActive() { return false; }
ncclResult_t groupDeferColl(const CollInfo&) { return ncclSuccess; }
void groupRecordError(ncclResult_t) {}
void tunerPick(ncclComm*, CollFunc, size_t, int, int, int, int*, int* nch) { *nch = 0; }
bool regCovers(ncclComm*, const void*, size_t) { return false; }
ncclResult_t commCheck(const ncclComm*, const char*, const char*) { return ncclSuccess; }
void commPollAsync(ncclComm*) {}
void ipcDrainReleases() {}
void ipcProgressReleases() {}
void regProgress(ncclComm*) {}
void regRecordUse(ncclComm*, const SymPlan&) {}
ncclResult_t bounceLaunch(ncclComm*, const SymPlan& sp) { return launchSymPlan(sp); }
void ipcNoteLaunch(hipStream_t, int) {}
bool ipcLibraryIdle() { return true; }
}  // namespace ncclamd

using namespace ncclamd;

int main(int argc, char** argv) {
  if (argc == 4 && !strcmp(argv[1], "peers")) {
    // the kernels' per-channel peer order (device_abi.h chanPeer): one line "me c p(1) ... p(n-1)" per (rank, channel)
    const int n = atoi(argv[2]), K = atoi(argv[3]);
    for (int me = 0; me < n; me++)
      for (int c = 0; c < K; c++) {
        printf("%d %d", me, c);
        for (int k = 1; k < n; k++) printf(" %d", chanPeer(me, n, c, k));
        printf("\n");
      }
    return 0;
  }
  if (argc == 4 && !strcmp(argv[1], "cap")) {  // the co-residency channel cap for (CUs, ranks per GPU)
    printf("%d\n", coResidentChannelCap(atoi(argv[2]), atoi(argv[3])));
    return 0;
  }
  if (argc == 2 && !strcmp(argv[1], "matrix")) {
    // NCCL_ALGO / NCCL_PROTO as loadTuning resolves them: "parse=<ncclResult_t>", then one line per collective
    CommTuning t;
    loadTuning(&t);
    printf("parse=%d\n", t.parseError);
    const char* fn[] = {"allreduce", "reducescatter", "allgather", "reduce"};
    const char* force[] = {"none", "oneshot", "direct", "ring", "tree"};
    for (int f = 0; f < FUNC_COUNT; f++) {
      const FuncTuning& ft = t.fn[f];
      printf("func=%s algo=%s oneshot=%d direct=%d noalgo=%d ll=%d ll128=%d simple=%d\n", fn[f], force[ft.algo],
             ft.oneShotOk, ft.directOk, ft.noAlgo, ft.llOn, ft.ll128On, ft.simpleOn);
    }
    return 0;
  }
  if (argc < 5) {
    fprintf(stderr, "usage: plan_test NRANKS FUNC DTYPE COUNT [ALIGN_OFFSET] [CHANCAP]\n");
    return 2;
  }
  const int n = atoi(argv[1]);
  const char* f = argv[2];
  const bool batch = !strcmp(f, "batch");
  const int dt = batch ? 0 : atoi(argv[3]);
  const size_t count = batch ? 0 : strtoull(argv[4], nullptr, 0);
  const size_t off = !batch && argc > 5 ? strtoull(argv[5], nullptr, 0) : 0;
  ncclComm comm;
  comm.startMagic = comm.endMagic = kCommMagic;
  comm.rank = 0;
  comm.nRanks = n;
  comm.device = 0;
  comm.minCTAs = 1;
  comm.maxCTAs = comm.maxChannels = 256;
  comm.nSlots = 2;
  // commDefaults' slot size: 1 GiB staging budget / (channels x 2 kinds x 2 slots x n), in [16 KiB, 1 MiB]
  comm.slotBytes = ((size_t)1 << 30) / (256 * 2 * 2 * (n > 1 ? n : 2));
  if (comm.slotBytes > ((size_t)1 << 20)) comm.slotBytes = (size_t)1 << 20;
  if (comm.slotBytes < ((size_t)16 << 10)) comm.slotBytes = (size_t)16 << 10;
  comm.chanCap = !batch && argc > 6 ? atoi(argv[6]) : 256;
  comm.devComm = (DevComm*)0x1000;
  // PLAN_MULTIPROCESS=1: the peers live in other processes, every one serving registrations (init.cc)
  comm.multiProcess = comm.regIpcAll = getenv("PLAN_MULTIPROCESS") && atoi(getenv("PLAN_MULTIPROCESS"));
  loadTuning(&comm.tune);
  resolveLinkChannels(&comm.tune, n, getenv("NCCL_MAX_CTAS") != nullptr);
  if (batch) {
    // the group.cc loop: plan in order, extend the open run while batchable, else launch it
    gBatchMode = true;
    std::vector<PlannedColl> run;
    for (int i = 3; i < argc; i++) {
      char fn[16] = {};
      int dtype = 7, op = 0;
      unsigned long long cnt = 0;
      if (sscanf(argv[i], "%15[^:]:%d:%llu:%d", fn, &dtype, &cnt, &op) < 3) return 2;
      PlannedColl pc;
      memset(&pc.info, 0, sizeof(pc.info));
      pc.info.func = !strcmp(fn, "rs") ? FUNC_REDUCESCATTER : !strcmp(fn, "ag") ? FUNC_ALLGATHER
                   : !strcmp(fn, "reduce") ? FUNC_REDUCE : FUNC_ALLREDUCE;
      pc.info.opName = fn;
      pc.info.sendbuff = (const void*)(0x10000000ull * (i + 1));
      pc.info.recvbuff = (void*)(0x10000000ull * (i + 1) + 0x8000000ull);
      pc.info.count = cnt;
      pc.info.datatype = (ncclDataType_t)dtype;
      pc.info.op = (ncclRedOp_t)op;
      pc.info.comm = &comm;
      if (planColl(pc.info, pc.p, pc.sp, &pc.kind) != ncclSuccess) return 1;
      if (!batchable(run, pc)) {
        if (!run.empty() && launchBatch(run) != ncclSuccess) return 1;
        run.clear();
      }
      run.push_back(pc);
    }
    if (!run.empty() && launchBatch(run) != ncclSuccess) return 1;
    return 0;
  }
  CollInfo info;
  memset(&info, 0, sizeof(info));
  info.func = !strcmp(f, "rs") ? FUNC_REDUCESCATTER : !strcmp(f, "ag") ? FUNC_ALLGATHER
            : !strcmp(f, "reduce") ? FUNC_REDUCE : FUNC_ALLREDUCE;
  info.opName = f;
  info.sendbuff = (const void*)(0x10000000ull + off);
  info.recvbuff = (void*)(0x20000000ull + off);
  info.count = count;
  info.datatype = (ncclDataType_t)dt;
  info.op = ncclSum;
  info.comm = &comm;
  info.stream = nullptr;
  ncclResult_t r = launchColl(info);
  if (r != ncclSuccess) {
    printf("error=%d\n", (int)r);
    return 1;
  }
  if (gKind == 1) {
    printf("algo=sym nch=%d part=%lu slice=0 steps=1 chunk=%lu\n", gSym.nChannels, (unsigned long)gSym.args.part,
           (unsigned long)gSym.args.chunk);
    return 0;
  }
  const char* const* names = kAlgoNames;
  const char* pipes[] = {"ring", "ring", "ring", "chain", "chain"};
  const LaunchPlan& p = gPlan;
  if (p.algo == ALGO_PIPE) {
    const unsigned sub = p.args.refSub ? p.args.refSub : 1;
    printf("algo=%s kind=%d nch=%d part=%lu slice=%lu steps=%d chunk=%lu cbdlo=%lu cbdhi=%lu refnch=%d sub=%u\n",
           pipes[p.pipeKind], p.pipeKind, p.nChannels, (unsigned long)p.args.part, (unsigned long)p.args.slice,
           p.args.nSteps, (unsigned long)p.args.chunk, (unsigned long)p.args.cbdLo, (unsigned long)p.args.cbdHi,
           p.nChannels / (int)sub, sub);
    return 0;
  }
  if (p.algo == ALGO_LL)
    printf("algo=%s nch=%d part=%lu slice=0 steps=1 chunk=%lu\n", p.ll.ops[0].proto == LLP_LL64 ? "ll128" : "ll",
           p.nChannels, (unsigned long)p.ll.ops[0].part,
           (unsigned long)p.ll.ops[0].chunk);
  else
    printf("algo=%s nch=%d part=%lu slice=%lu steps=%d chunk=%lu cbdlo=%lu cbdhi=%lu refnch=%d sub=%u\n",
           names[p.algo], p.nChannels, (unsigned long)p.args.part, (unsigned long)p.args.slice, p.args.nSteps,
           (unsigned long)p.args.chunk, (unsigned long)p.args.cbdLo, (unsigned long)p.args.cbdHi,
           p.nChannels / (int)(p.args.refSub ? p.args.refSub : 1), p.args.refSub ? p.args.refSub : 1);
  return 0;
}
