// user_object_probe.hip — does a hipUserObject retained by a captured graph outlive hipGraphDestroy while an
// executable graph instantiated from it exists (CUDA's semantics), and when does its destructor run? Decides whether
// graph auto-registrations (register.cc, NCCL_GRAPH_REGISTER) can be tied to the graph's lifetime: PyTorch destroys
// the hipGraph_t right after instantiating it. Diagnostics only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <thread>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static std::atomic<int> gDestroyed{0};
static void destroyFn(void* p) { gDestroyed.fetch_add(1 + 0 * (int)(intptr_t)p); }

__global__ void bump(int* x) { x[0] += 1; }

static int waitDestroyed(int want, int ms) {
  for (int i = 0; i < ms && gDestroyed.load() < want; i++) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  return gDestroyed.load();
}

int main() {
  int* x;
  CK(hipMalloc(&x, sizeof(int)));
  CK(hipMemset(x, 0, sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // capture, retaining a user object on the capturing graph (what a library does from inside a captured call)
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(bump, dim3(1), dim3(1), 0, s, x);
  hipStreamCaptureStatus st;
  unsigned long long id = 0;
  hipGraph_t capGraph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nDeps = 0;
  CK(hipStreamGetCaptureInfo_v2(s, &st, &id, &capGraph, &deps, &nDeps));
  hipUserObject_t obj;
  CK(hipUserObjectCreate(&obj, (void*)0x1, destroyFn, 1, hipUserObjectNoDestructorSync));
  CK(hipGraphRetainUserObject(capGraph, obj, 1, hipGraphUserObjectMove));
  hipGraph_t g;
  CK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  CK(hipDeviceSynchronize());
  const int afterGraphDestroy = waitDestroyed(1, 200);
  for (int i = 0; i < 3; i++) CK(hipGraphLaunch(ex, s));
  CK(hipStreamSynchronize(s));
  const int afterReplays = waitDestroyed(1, 50);
  CK(hipGraphExecDestroy(ex));
  CK(hipDeviceSynchronize());
  const int afterExecDestroy = waitDestroyed(1, 2000);
  int h = 0;
  CK(hipMemcpy(&h, x, sizeof(int), hipMemcpyDeviceToHost));
  printf("{\"destroyed_after_graph_destroy\": %d, \"destroyed_after_replays\": %d, \"destroyed_after_exec_destroy\": %d, "
         "\"replays_ran\": %d}\n", afterGraphDestroy, afterReplays, afterExecDestroy, h);
  return 0;
}
