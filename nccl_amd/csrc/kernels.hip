// kernels.hip — nRanks==1 streaming copy kernels and the host-side launch dispatch.
// The collective kernels (kernels.h) are instantiated per element type in kern_<type>.hip.
#include <cxxabi.h>

#include <mutex>
#include <set>

#include "kernels.h"

namespace ncclamd {

ncclResult_t launchKernU8(const LaunchPlan& p);
ncclResult_t launchKernU32(const LaunchPlan& p);
ncclResult_t launchKernU64(const LaunchPlan& p);
ncclResult_t launchKernF16(const LaunchPlan& p);
ncclResult_t launchKernBF16(const LaunchPlan& p);
ncclResult_t launchKernF32(const LaunchPlan& p);
ncclResult_t launchKernF64(const LaunchPlan& p);
ncclResult_t launchKernFp8(const LaunchPlan& p);
ncclResult_t launchKernGather(const LaunchPlan& p);
ncclResult_t launchSymKernU8(const SymPlan& p);
ncclResult_t launchSymKernU32(const SymPlan& p);
ncclResult_t launchSymKernU64(const SymPlan& p);
ncclResult_t launchSymKernF16(const SymPlan& p);
ncclResult_t launchSymKernBF16(const SymPlan& p);
ncclResult_t launchSymKernF32(const SymPlan& p);
ncclResult_t launchSymKernF64(const SymPlan& p);
ncclResult_t launchSymKernFp8(const SymPlan& p);
ncclResult_t launchSymKernGather(const SymPlan& p);
hipError_t warmKernU8();
hipError_t warmKernU32();
hipError_t warmKernU64();
hipError_t warmKernF16();
hipError_t warmKernBF16();
hipError_t warmKernF32();
hipError_t warmKernF64();
hipError_t warmKernFp8();
hipError_t warmKernGather();

// Load every kernel code object of this library on the current device at communicator init. With
// lazy code-object loading, the first launch of a kernel from a not-yet-loaded object may wait for
// the device to go idle; when several ranks share one GPU inside one process (ncclCommInitAll with a
// repeated device) the peer rank's already-running, spinning kernel would then never see its partner
// launch. Loading up front removes that stall from the collective launch path.
ncclResult_t warmKernels() {
  hipError_t (*fns[])() = {warmKernU8, warmKernU32, warmKernU64, warmKernF16, warmKernBF16,
                           warmKernF32, warmKernF64, warmKernFp8, warmKernGather};
  for (auto f : fns) HIPCHECK(f());
  return ncclSuccess;
}

// ------------------------------------------------------------------------------------ kernel log

bool gKernelLog = getenv("NCCL_AMD_KERNEL_LOG") != nullptr;

void kernelLogNote(const void* fn, unsigned grid, unsigned block) {
  static std::mutex mu;
  static std::set<std::pair<const void*, unsigned>> seen;
  std::lock_guard<std::mutex> g(mu);
  if (!seen.insert({fn, grid}).second) return;
  const char* raw = hipKernelNameRefByPtr(fn, nullptr);
  int st = -1;
  char* dem = raw ? abi::__cxa_demangle(raw, nullptr, nullptr, &st) : nullptr;
  if (FILE* f = fopen(getenv("NCCL_AMD_KERNEL_LOG"), "a")) {
    fprintf(f, "%s grid=%u block=%u\n", st == 0 && dem ? dem : raw ? raw : "?", grid, block);
    fclose(f);
  }
  free(dem);
}

// ------------------------------------------------------------------------------------ nRanks == 1


// Streaming copy (reference onerank.cu:52-56 uses cudaMemcpyAsync; this is the hand-written
// replacement): 16 B per lane, U packs in flight per lane, grid-stride over 256*U*16-byte tiles.
// NTL selects nontemporal loads; SPOL the store: -2 plain, -1 global nontemporal, >= 0 a buffer store with
// that cache policy (sc0 = 1, nt = 2, sc1 = 16; offsets from the tile's own base, so 32 bits suffice)
// (measured variants). XCD: the dispatcher hands workgroup b to XCD b % 8, so with the identity
// mapping every XCD streams every eighth tile; instead the tiles are permuted so that each XCD streams runs of
// 2^kshift consecutive tiles (the grid's last G % (8 << kshift) workgroups keep their own tile). Default 2^6 tiles
// (512 KiB per XCD, 4 MiB per round): bench N=1 frac 0.911-0.916 warm, 0.798-0.807 cold vs 0.899-0.906 / 0.792-0.800
// for the identity mapping; runs of 2^3-2^5 and 2^10-2^12 tiles were no better (profiles/r04_copy_xcd_shift_ab.txt).
template <int U, bool NTL, int SPOL, bool XCD = false>
__global__ void __launch_bounds__(256) copyKernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                  uint64_t npk, uint32_t kshift) {
  uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  uint64_t tile = blockIdx.x;
  if constexpr (XCD) {
    // rounds of 8 * 2^kshift tiles: XCD x takes the x-th run of 2^kshift consecutive tiles of each round
    const uint32_t grp = 8u << kshift, j = blockIdx.x >> 3, x = blockIdx.x & 7;
    if (blockIdx.x < gridDim.x / grp * grp) tile = (uint64_t)(j >> kshift) * grp + (x << kshift) + (j & ((1u << kshift) - 1));
  }
  for (uint64_t t0 = tile * 256 * U; t0 < npk; t0 += stride) {
    const uint64_t base = t0 + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * 256 < npk) v[u] = NTL ? __builtin_nontemporal_load(src + base + u * 256) : src[base + u * 256];
    __amdgpu_buffer_rsrc_t rd;
    if constexpr (SPOL >= 0) rd = remoteRsrc(dst + t0);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * 256 < npk) {
        if constexpr (SPOL >= 0) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (uint32_t)((threadIdx.x + u * 256) * 16), 0, SPOL);
        else if constexpr (SPOL == -1) __builtin_nontemporal_store(v[u], dst + base + u * 256);
        else dst[base + u * 256] = v[u];
      }
  }
}

__global__ void copyBytesKernel(char* dst, const char* src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

ncclResult_t launchCopy(void* dst, const void* src, size_t bytes, hipStream_t stream, int var, int64_t gridCap,
                        int xcdShift) {
  if (bytes == 0 || dst == src) return ncclSuccess;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    uint64_t npk = bytes >> 4;
    if (npk) {
      // variant (NCCL_AMD_COPY_VARIANT): 0 (default) nt loads + system-scope write-through buffer stores
      // (sc0|sc1), 2 packs per thread (8 KiB tiles), tiles mapped XCD-contiguous; 10 the same with the identity
      // tile mapping (the round-3 default); 11 / 12 the default with 4 / 1 packs per thread; 1 plain/plain U4, 2 plain/global-nt U4, 3 nt/global-nt U8, 9 nt/global-nt
      // U4 (the round-1/2 default); nt loads with U4 buffer stores under cache policy 4 sc0|sc1, 5 sc1, 6 sc1|nt,
      // 7 nt, 8 none (scripts/copy_policy_probe.hip, copy_shape_probe.hip, load_policy_probe.hip)
      int U = var == 3 ? 8 : var == 12 ? 1 : (var == 0 || var == 10 || var > 12) ? 2 : 4;
      uint64_t tiles = (npk + 256 * U - 1) / (256 * U);
      // one 16 KiB tile per workgroup by default: measured best on 256 MiB with buffers rotated past the
      // 256 MiB Infinity Cache (6.48 TB/s vs 6.26 for a 2048-block grid-stride; scripts/copy_variants.hip)
      int grid = (int)std::min<uint64_t>(tiles, (uint64_t)(gridCap > 0 ? gridCap : 1));
      // the XCD runs: 2^xcdShift tiles (NCCL_AMD_COPY_XCD_SHIFT), capped at an eighth of the grid
      uint32_t xshift = (uint32_t)std::max(0, xcdShift);
      while (xshift > 0 && ((uint64_t)8 << xshift) > (uint64_t)grid) xshift--;
      u32x4* d = (u32x4*)dst;
      const u32x4* s = (const u32x4*)src;
      switch (var) {
        case 1: NCCL_AMD_LAUNCH((copyKernel<4, false, -2>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 2: NCCL_AMD_LAUNCH((copyKernel<4, false, -1>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 3: NCCL_AMD_LAUNCH((copyKernel<8, true, -1>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 5: NCCL_AMD_LAUNCH((copyKernel<4, true, 16>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 6: NCCL_AMD_LAUNCH((copyKernel<4, true, 18>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 7: NCCL_AMD_LAUNCH((copyKernel<4, true, 2>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 8: NCCL_AMD_LAUNCH((copyKernel<4, true, 0>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 9: NCCL_AMD_LAUNCH((copyKernel<4, true, -1>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 4: NCCL_AMD_LAUNCH((copyKernel<4, true, 17>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 10: NCCL_AMD_LAUNCH((copyKernel<2, true, 17>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 11: NCCL_AMD_LAUNCH((copyKernel<4, true, 17, true>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        case 12: NCCL_AMD_LAUNCH((copyKernel<1, true, 17, true>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
        default: NCCL_AMD_LAUNCH((copyKernel<2, true, 17, true>), dim3(grid), dim3(256), 0, stream, d, s, npk, xshift); break;
      }
      HIPCHECK(hipGetLastError());
    }
    uint64_t done = npk << 4;
    if (done < bytes) {
      NCCL_AMD_LAUNCH(copyBytesKernel, dim3(1), dim3(64), 0, stream, (char*)dst + done, (const char*)src + done,
                         (uint64_t)(bytes - done));
      HIPCHECK(hipGetLastError());
    }
    return ncclSuccess;
  }
  int grid = (int)std::min<uint64_t>(2048, (bytes + 255) / 256);
  NCCL_AMD_LAUNCH(copyBytesKernel, dim3(grid), dim3(256), 0, stream, (char*)dst, (const char*)src, (uint64_t)bytes);
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

// ------------------------------------------------------------------------------------ mapping check (mapcheck.cc)

// One wave: lane p (a peer) stores the pattern (me -> p) into p's staging slot [0][RS][0][me] and flag probe row 0
// [me] through this rank's mapping of p — 16-byte system-scope write-through stores, the collective kernels' own
// remote-store flavour — and loads p's self patterns (staging slot [0][AG][0][p], probe row 1) through the same
// mappings, with the flag loads' system scope, into out[p][0..3]. skip (tests): no remote stores, as a mapping that
// drops them would.
__global__ void __launch_bounds__(64) mapCheckKernel(const DevComm* dcp, MapCheckArgs a, uint64_t* out) {
  const DevComm& dc = *dcp;
  const int p = threadIdx.x, me = dc.rank;
  if (p < dc.nRanks && p != me) {
    const uint64_t slotW = stagingOffset(dc, 0, STG_RS, 0, me), slotR = stagingOffset(dc, 0, STG_AG, 0, p);
    char* fl = (char*)dc.flags[p] + a.probeOff;
    if (!a.skip) {
      u32x4 v0, v1;
      __builtin_memcpy(&v0, a.w[p][0], 16);
      __builtin_memcpy(&v1, a.w[p][1], 16);
      storeRemote(dc.staging[p] + slotW, v0);
      storeRemote(fl + (size_t)me * 16, v1);
    }
    const uint64_t* rs = (const uint64_t*)(dc.staging[p] + slotR);
    const uint64_t* rf = (const uint64_t*)(fl + NCCL_AMD_MAX_RANKS * 16);
    out[p * 4 + 0] = loadFlag(rs);
    out[p * 4 + 1] = loadFlag(rs + 1);
    out[p * 4 + 2] = loadFlag(rf);
    out[p * 4 + 3] = loadFlag(rf + 1);
  }
  drainStores();
}

ncclResult_t launchMapCheck(const DevComm* dc, const MapCheckArgs& a, uint64_t* out, hipStream_t stream) {
  NCCL_AMD_LAUNCH(mapCheckKernel, dim3(1), dim3(64), 0, stream, dc, a, out);
  HIPCHECK(hipGetLastError());
  return ncclSuccess;
}

ncclResult_t launchPlan(const LaunchPlan& p) {
  if (p.algo == ALGO_COPY)
    return launchCopy(p.args.recvbuff, p.args.sendbuff, p.bytes, p.stream, p.copyVariant, p.copyGrid, p.copyXcdShift);
  if (p.func == FUNC_ALLGATHER) return launchKernGather(p);
  switch (p.datatype) {
    case ncclInt8: case ncclUint8: return launchKernU8(p);
    case ncclInt32: case ncclUint32: return launchKernU32(p);
    case ncclInt64: case ncclUint64: return launchKernU64(p);
    case ncclFloat16: return launchKernF16(p);
    case ncclBfloat16: return launchKernBF16(p);
    case ncclFloat32: return launchKernF32(p);
    case ncclFloat64: return launchKernF64(p);
    case ncclFloat8e4m3: case ncclFloat8e5m2: return launchKernFp8(p);
    default: break;
  }
  return ncclInvalidArgument;
}

ncclResult_t launchSymPlan(const SymPlan& p) {
  if (p.coll == SYM_AG) return launchSymKernGather(p);
  switch (p.datatype) {
    case ncclInt8: case ncclUint8: return launchSymKernU8(p);
    case ncclInt32: case ncclUint32: return launchSymKernU32(p);
    case ncclInt64: case ncclUint64: return launchSymKernU64(p);
    case ncclFloat16: return launchSymKernF16(p);
    case ncclBfloat16: return launchSymKernBF16(p);
    case ncclFloat32: return launchSymKernF32(p);
    case ncclFloat64: return launchSymKernF64(p);
    case ncclFloat8e4m3: case ncclFloat8e5m2: return launchSymKernFp8(p);
    default: break;
  }
  return ncclInvalidArgument;
}

}  // namespace ncclamd
