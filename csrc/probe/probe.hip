// HIP/CDNA4 link-cost probe kernels (gfx950) + pybind11 bindings.
//
// Reference: design.md:23-59 obtains the GPU-pair link class from NVML and leaves the bandwidth
// weight as a TODO (design.md:47).  On MI355X every GPU pair is a direct xGMI link, so the link
// class alone cannot rank placements; instead the device plugin measures the real link-cost matrix
// at node start with the kernels below:
//   K1 p2p read  : kernel on the reader GPU pulls a peer buffer over xGMI, staged through LDS by
//                  LDS-DMA (global_load_lds_dwordx4) and stored to local HBM.
//   K2 p2p write : kernel on the source GPU pushes local HBM into the peer buffer.
//   K3 hbm copy  : self pair (k=1 baseline), same kernel with both pointers local.
//   K4 mfma warm : v_mfma_f32_32x32x16_bf16 loop to lift clocks before timing, also reporting the
//                  achieved dense bf16 rate.
//   K5 gather    : one kernel on the reader pulls from all of its peers at once -> aggregate xGMI
//                  ingress per GPU with every other GPU idle.
//   K6 ring      : every member of a subset runs the K5 gather from its peers at the same time
//                  (ingress and egress of every GPU loaded together, as under a ring all-reduce):
//                  the slowest member's ingress is the bound a ring all-reduce's busBW is measured
//                  against.
//   IPC read     : the K1 kernel on a buffer another process exported with hipIpcGetMemHandle (the
//                  mapping RCCL's P2P transport gives a rank of its peers' buffers).
// The copy kernel exists in two staging forms (LDS-DMA and plain register staging) so the
// rocprofv3 counter profile can show what LDS staging costs/buys on a pure stream (profiles/).
//
// Geometry (CDNA4): 256-thread blocks (4 wave64), each wave moves 64 lanes x 16 B = 1 KiB per
// instruction; UNROLL=4 instructions in flight per lane -> 16 KiB LDS image per block, so up to
// 8 blocks (32 waves, the CU maximum) are resident per CU inside the 160 KiB LDS.  Grid = CUs x 8
// with a grid-stride loop: >>256 workgroups fills all 8 XCDs; a streaming copy has no reuse so no
// XCD remap is needed (each byte is touched once).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HIP_CHECK(expr)                                                                          \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess)                                                                        \
      throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                       \
  } while (0)

namespace {

constexpr int kBlock = 256;
constexpr int kUnroll = 4;
constexpr int kTileVec = kBlock * kUnroll;  // 16-byte vectors per block-iteration (16 KiB)
constexpr int kBlocksPerCU = 8;

using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;

// ---------------------------------------------------------------------------------------------
// K1/K2/K3: LDS-DMA staged copy.  Each wave issues kUnroll global_load_lds_dwordx4 into its own
// 1 KiB LDS slices (wave-uniform base + lane*16: the DMA's lane-linear rule), drains vmcnt, then
// each lane stores back the 16 B its own lane fetched, so no cross-wave barrier is needed.
// `blk`/`nblk` let one launch split its grid over several streams (K5 gather below).
template <bool kNonTemporal>
__device__ __forceinline__ void copy_lds_stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n_vec,
                                                u32x4* lds, size_t blk, size_t nblk) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const size_t n_full = (n_vec / kTileVec) * kTileVec;
  for (size_t base = blk * kTileVec; base < n_full; base += nblk * kTileVec) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const size_t off = base + (size_t)u * kBlock + wave * 64;
      __builtin_amdgcn_global_load_lds((gptr_t)(src + off + lane), (lptr_t)(lds + u * kBlock + wave * 64), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const size_t off = base + (size_t)u * kBlock + wave * 64 + lane;
      u32x4 v = lds[u * kBlock + wave * 64 + lane];
      if (kNonTemporal)
        __builtin_nontemporal_store(v, dst + off);
      else
        dst[off] = v;
    }
  }
  // tail (< one tile): plain per-thread copy
  for (size_t i = n_full + blk * kBlock + threadIdx.x; i < n_vec; i += nblk * kBlock) dst[i] = src[i];
}

template <bool kNonTemporal>
__global__ __launch_bounds__(kBlock) void copy_lds_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                          size_t n_vec) {
  __shared__ u32x4 lds[kTileVec];
  copy_lds_stream<kNonTemporal>(src, dst, n_vec, lds, blockIdx.x, gridDim.x);
}

// K5 gather: one launch on the reader pulls from up to kMaxSrc peers at once (ingress over all of
// its xGMI links together).  Block b serves source b % nsrc, so every source gets gridDim/nsrc
// blocks spread over all XCDs; source s lands in dst[s * n_vec ...].
constexpr int kMaxSrc = 16;
struct SrcSet {
  const u32x4* p[kMaxSrc];
};

__global__ __launch_bounds__(kBlock) void gather_lds_kernel(SrcSet srcs, int nsrc, u32x4* __restrict__ dst,
                                                            size_t n_vec) {
  __shared__ u32x4 lds[kTileVec];
  const int s = blockIdx.x % nsrc;
  copy_lds_stream<true>(srcs.p[s], dst + (size_t)s * n_vec, n_vec, lds, blockIdx.x / nsrc, gridDim.x / nsrc);
}

// Register-staged variant of the same stream (kUnroll independent 16-B loads in flight per lane).
template <bool kNonTemporal>
__global__ __launch_bounds__(kBlock) void copy_reg_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                          size_t n_vec) {
  const size_t n_full = (n_vec / kTileVec) * kTileVec;
  for (size_t base = (size_t)blockIdx.x * kTileVec; base < n_full; base += (size_t)gridDim.x * kTileVec) {
    u32x4 r[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) r[u] = src[base + (size_t)u * kBlock + threadIdx.x];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (kNonTemporal)
        __builtin_nontemporal_store(r[u], dst + base + (size_t)u * kBlock + threadIdx.x);
      else
        dst[base + (size_t)u * kBlock + threadIdx.x] = r[u];
    }
  }
  for (size_t i = n_full + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n_vec; i += (size_t)gridDim.x * kBlock)
    dst[i] = src[i];
}

// Contiguous-chunk variant: block b streams its own 1/grid slice of the buffer (each workgroup walks
// one DRAM region, instead of the whole grid sweeping one window together), U independent 16-B
// loads in flight per lane, non-temporal loads and stores.
template <int U>
__global__ __launch_bounds__(kBlock) void copy_chunk_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                            size_t n_vec) {
  const size_t tile = (size_t)kBlock * U;
  const size_t n_tiles = n_vec / tile;
  const size_t per = (n_tiles + gridDim.x - 1) / gridDim.x;
  const size_t t0 = (size_t)blockIdx.x * per;
  const size_t t1 = std::min(n_tiles, t0 + per);
  for (size_t t = t0; t < t1; ++t) {
    const size_t base = t * tile + threadIdx.x;
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(src + base + (size_t)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + base + (size_t)u * kBlock);
  }
  for (size_t i = n_tiles * tile + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n_vec; i += (size_t)gridDim.x * kBlock)
    dst[i] = src[i];
}

__global__ __launch_bounds__(kBlock) void fill_pattern_kernel(unsigned int* __restrict__ p, size_t n_words,
                                                              unsigned int seed) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n_words; i += (size_t)gridDim.x * kBlock)
    p[i] = (unsigned int)(i * 2654435761u) ^ seed;
}

// K4: MFMA warm-up.  Each wave keeps 4 independent 32x32 accumulators so back-to-back
// v_mfma_f32_32x32x16_bf16 issue is not serialised on the dependent-accumulator latency.
__global__ __launch_bounds__(kBlock) void mfma_warmup_kernel(float* __restrict__ out, int iters) {
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)((threadIdx.x & 7) * 0.125f - 0.5f);
    b[i] = (__bf16)(i * 0.0625f - 0.25f);
  }
  f32x16 acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
  for (int it = 0; it < iters; ++it) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
  out[(size_t)blockIdx.x * kBlock + threadIdx.x] = s;
}

// K4r: the same loop on random operands.  Eight distinct pseudo-random A and B fragments per lane
// (uniform in [-1, 1), from a hash of lane and index) are cycled, so consecutive MFMAs see new
// operand bits as a GEMM's do.  The bit toggling draws more power than K4's near-constant operands;
// the rate it reaches is the MFMA ceiling a GEMM or an attention kernel on real data can approach.
__device__ __forceinline__ __bf16 rand_bf16(unsigned int x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return (__bf16)((float)(x >> 8) * (1.0f / 8388608.0f) - 1.0f);
}

__global__ __launch_bounds__(kBlock) void mfma_warmup_random_kernel(float* __restrict__ out, int iters) {
  bf16x8 a[8], b[8];
  const unsigned int seed = (blockIdx.x * kBlock + threadIdx.x) * 131u;
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[f][i] = rand_bf16(seed + 16u * f + i);
      b[f][i] = rand_bf16(~(seed + 16u * f + i));
    }
  f32x16 acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
  for (int it = 0; it < iters; it += 2) {
#pragma unroll
    for (int f = 0; f < 8; f += 4) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f], b[f + 1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 1], b[f + 2], acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 2], b[f + 3], acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 3], b[f], acc3, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + acc2[i] + acc3[i];
  out[(size_t)blockIdx.x * kBlock + threadIdx.x] = s;
}

// Where a workgroup runs: its XCD (HW_REG_XCC_ID[3:0]) and the low half of HW_REG_HW_ID (wave, SIMD,
// CU, SH, SE).  Lane 0 writes one word per workgroup with an ordinary vector store.  Shows how a queue
// CU mask (HSA_CU_MASK, time-sliced shares in topology/shares.py) spreads over the 8 XCDs.
__global__ __launch_bounds__(64) void xcc_census_kernel(unsigned int* __restrict__ out) {
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu;  // hwreg(HW_REG_XCC_ID, 0, 4)
  const unsigned hw = __builtin_amdgcn_s_getreg((15 << 11) | 4);          // hwreg(HW_REG_HW_ID, 0, 16)
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc << 16) | (hw & 0xFFFFu);
}

// ---------------------------------------------------------------------------------------------
struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    HIP_CHECK(hipGetDevice(&prev));
    HIP_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

struct DevBuf {
  void* p = nullptr;
  int dev = -1;
  size_t bytes = 0;
  DevBuf(int d, size_t b) : dev(d), bytes(b) {
    DeviceGuard g(d);
    HIP_CHECK(hipMalloc(&p, b));
  }
  ~DevBuf() {
    if (p) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      (void)hipSetDevice(prev);
    }
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

int num_cus(int dev) {
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return std::max(cus, 1);
}

void enable_peer(int from, int to) {
  if (from == to) return;
  int can = 0;
  HIP_CHECK(hipDeviceCanAccessPeer(&can, from, to));
  if (!can) throw std::runtime_error("device " + std::to_string(from) + " cannot access peer " + std::to_string(to));
  DeviceGuard g(from);
  hipError_t e = hipDeviceEnablePeerAccess(to, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
    throw std::runtime_error(std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
  (void)hipGetLastError();
}

void launch_copy(const std::string& kind, bool nt, const void* src, void* dst, size_t n_vec, int grid, hipStream_t s) {
  auto* S = reinterpret_cast<const u32x4*>(src);
  auto* D = reinterpret_cast<u32x4*>(dst);
  if (kind == "lds") {
    if (nt)
      hipLaunchKernelGGL(copy_lds_kernel<true>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
    else
      hipLaunchKernelGGL(copy_lds_kernel<false>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
  } else if (kind == "reg") {
    if (nt)
      hipLaunchKernelGGL(copy_reg_kernel<true>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
    else
      hipLaunchKernelGGL(copy_reg_kernel<false>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
  } else if (kind == "chunk") {
    hipLaunchKernelGGL(copy_chunk_kernel<8>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
  } else if (kind == "chunk4") {
    hipLaunchKernelGGL(copy_chunk_kernel<4>, dim3(grid), dim3(kBlock), 0, s, S, D, n_vec);
  } else if (kind == "sdma") {
    HIP_CHECK(hipMemcpyAsync(dst, src, n_vec * 16, hipMemcpyDeviceToDevice, s));
    return;
  } else {
    throw std::invalid_argument("kind must be lds|reg|chunk|chunk4|sdma");
  }
  HIP_CHECK(hipGetLastError());
}

// Verify a few windows of dst against the host-side pattern.
bool verify_pattern(const DevBuf& dst, size_t n_words, unsigned int seed) {
  const size_t win = std::min<size_t>(n_words, 1 << 16);
  std::vector<size_t> starts = {0, n_words / 2 - std::min(n_words / 2, win / 2), n_words - win};
  std::vector<unsigned int> h(win);
  DeviceGuard g(dst.dev);
  for (size_t st : starts) {
    HIP_CHECK(hipMemcpy(h.data(), (const unsigned int*)dst.p + st, win * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < win; ++i) {
      unsigned int want = (unsigned int)((st + i) * 2654435761u) ^ seed;
      if (h[i] != want) return false;
    }
  }
  return true;
}

struct CopyResult {
  int src, dst, exec, iters, grid;
  size_t bytes;
  std::string kind;
  bool nontemporal, ok;
  double ms_per_iter, gbps;
};

CopyResult copy_bw_impl(int src_dev, int dst_dev, int exec_dev, size_t bytes, int iters, int warmup,
                        const std::string& kind, bool nontemporal, int blocks_per_cu) {
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (exec_dev != src_dev && exec_dev != dst_dev) throw std::invalid_argument("exec_dev must be src or dst");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  for (int d : {src_dev, dst_dev})
    if (d < 0 || d >= ndev) throw std::invalid_argument("device index out of range");
  if (src_dev != dst_dev) enable_peer(exec_dev, exec_dev == src_dev ? dst_dev : src_dev);

  DevBuf src(src_dev, bytes), dst(dst_dev, bytes);
  const size_t n_vec = bytes / 16;
  const unsigned int seed = 0x9e3779b9u ^ (unsigned)(src_dev * 131 + dst_dev);
  {
    DeviceGuard g(src_dev);
    hipLaunchKernelGGL(fill_pattern_kernel, dim3(num_cus(src_dev) * 4), dim3(kBlock), 0, 0, (unsigned int*)src.p,
                       bytes / 4, seed);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
  }
  DeviceGuard g(exec_dev);
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int grid = num_cus(exec_dev) * std::max(1, blocks_per_cu);
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  float ms = 0.f;
  try {
    for (int i = 0; i < warmup; ++i) launch_copy(kind, nontemporal, src.p, dst.p, n_vec, grid, s);
    HIP_CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) launch_copy(kind, nontemporal, src.p, dst.p, n_vec, grid, s);
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipEventSynchronize(e1));
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  } catch (...) {
    (void)hipStreamSynchronize(s);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    throw;
  }
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  HIP_CHECK(hipStreamDestroy(s));
  const bool ok = verify_pattern(dst, bytes / 4, seed);
  const double sec = ms / 1e3 / iters;
  // gbps = bytes copied per second (one direction over the link; for a self copy HBM moves 2x)
  return CopyResult{src_dev, dst_dev, exec_dev, iters, grid, bytes, kind, nontemporal, ok, (double)ms / iters,
                    (double)bytes / sec / 1e9};
}

// K5: aggregate ingress of `dst_dev` reading `bytes` from every device in `srcs` concurrently.
// A source equal to dst_dev is a local stream (one buffer per entry), which lets a 1-GPU box check
// the kernel's segment indexing; on a node the sources are the peers.
py::dict gather_bw(int dst_dev, const std::vector<int>& srcs, size_t bytes, int iters, int warmup, int blocks_per_cu) {
  if (srcs.empty() || srcs.size() > (size_t)kMaxSrc) throw std::invalid_argument("1..16 source devices");
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  if (dst_dev < 0 || dst_dev >= ndev) throw std::invalid_argument("device index out of range");
  for (int d : srcs) {
    if (d < 0 || d >= ndev) throw std::invalid_argument("source device index out of range");
  }
  double ms_total = 0.0;
  bool ok = true;
  const int nsrc = (int)srcs.size();
  {
    py::gil_scoped_release nogil;
    for (int d : srcs) enable_peer(dst_dev, d);
    std::vector<std::unique_ptr<DevBuf>> src_bufs;
    SrcSet set{};
    for (int i = 0; i < nsrc; ++i) {
      src_bufs.emplace_back(new DevBuf(srcs[i], bytes));
      DeviceGuard g(srcs[i]);
      hipLaunchKernelGGL(fill_pattern_kernel, dim3(num_cus(srcs[i]) * 4), dim3(kBlock), 0, 0,
                         (unsigned int*)src_bufs.back()->p, bytes / 4, 0x51ed27u ^ (unsigned)(srcs[i] * 977));
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipDeviceSynchronize());
      set.p[i] = reinterpret_cast<const u32x4*>(src_bufs.back()->p);
    }
    DevBuf dst(dst_dev, bytes * (size_t)nsrc);
    DeviceGuard g(dst_dev);
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int per = std::max(1, num_cus(dst_dev) * std::max(1, blocks_per_cu) / nsrc);
    const int grid = per * nsrc;  // a multiple of nsrc: every source gets the same block count
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (int i = 0; i < warmup; ++i)
      hipLaunchKernelGGL(gather_lds_kernel, dim3(grid), dim3(kBlock), 0, st, set, nsrc, (u32x4*)dst.p, bytes / 16);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i)
      hipLaunchKernelGGL(gather_lds_kernel, dim3(grid), dim3(kBlock), 0, st, set, nsrc, (u32x4*)dst.p, bytes / 16);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(e1, st));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms_total = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    // verify every segment against its source's pattern (windows, as for the pairwise probe)
    const size_t words = bytes / 4, win = std::min<size_t>(words, 1 << 14);
    std::vector<unsigned int> h(win);
    for (int i = 0; i < nsrc && ok; ++i) {
      const unsigned int seed = 0x51ed27u ^ (unsigned)(srcs[i] * 977);
      for (size_t st0 : {(size_t)0, words - win}) {
        HIP_CHECK(hipMemcpy(h.data(), (const unsigned int*)dst.p + (size_t)i * words + st0, win * 4, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < win; ++k)
          if (h[k] != ((unsigned int)((st0 + k) * 2654435761u) ^ seed)) {
            ok = false;
            break;
          }
      }
    }
  }
  const double sec = ms_total / 1e3 / iters;
  py::dict r;
  r["dst"] = dst_dev;
  r["srcs"] = srcs;
  r["bytes_per_src"] = bytes;
  r["iters"] = iters;
  r["ms_per_iter"] = ms_total / iters;
  r["gbps"] = (double)bytes * nsrc / sec / 1e9;
  r["ok"] = ok;
  return r;
}

// K6 ring: every member of a subset gathers from its peers AT THE SAME TIME, so each GPU's xGMI
// ingress and egress are loaded together, as they are under a ring all-reduce (K1 loads one
// direction of one idle link; K5 loads one GPU's ingress with every other GPU idle).  Member m runs
// the K5 gather kernel on its own stream of devs[m], pulling the source buffer of every member in
// peers[m] into its own inbox; launches are interleaved across members so they overlap from the
// first iteration.  A member's rate is the bytes it received / its own stream time; the subset's
// ring bound is the slowest member (a ring all-reduce's busBW is every member's ingress rate, so
// the slowest one caps it).  Members may repeat a device: on one GPU that checks the indexing.
py::dict ring_bw(const std::vector<int>& devs, const std::vector<std::vector<int>>& peers, size_t bytes, int iters,
                 int warmup, int blocks_per_cu) {
  const int k = (int)devs.size();
  if (k < 2 || k > kMaxSrc + 1) throw std::invalid_argument("2..17 ring members");
  if ((int)peers.size() != k) throw std::invalid_argument("one peer list per member");
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  for (int d : devs)
    if (d < 0 || d >= ndev) throw std::invalid_argument("device index out of range");
  for (int m = 0; m < k; ++m) {
    if (peers[m].empty() || peers[m].size() > (size_t)kMaxSrc) throw std::invalid_argument("1..16 peers per member");
    for (int p : peers[m])
      if (p < 0 || p >= k || p == m) throw std::invalid_argument("peers are other members' indices");
  }
  auto seed_of = [](int m) { return 0x6a09e667u ^ (unsigned)(m * 7919 + 1); };
  std::vector<double> ms_member(k, 0.0);
  double wall_ms = 0.0;
  bool ok = true;
  {
    py::gil_scoped_release nogil;
    for (int m = 0; m < k; ++m)
      for (int p : peers[m]) enable_peer(devs[m], devs[p]);
    std::vector<std::unique_ptr<DevBuf>> src, inbox;
    for (int m = 0; m < k; ++m) {
      src.emplace_back(new DevBuf(devs[m], bytes));
      inbox.emplace_back(new DevBuf(devs[m], bytes * peers[m].size()));
      DeviceGuard g(devs[m]);
      hipLaunchKernelGGL(fill_pattern_kernel, dim3(num_cus(devs[m]) * 4), dim3(kBlock), 0, 0, (unsigned int*)src[m]->p,
                         bytes / 4, seed_of(m));
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipDeviceSynchronize());
    }
    std::vector<SrcSet> sets(k);
    std::vector<int> grid(k);
    std::vector<hipStream_t> st(k, nullptr);
    std::vector<hipEvent_t> e0(k, nullptr), e1(k, nullptr);
    for (int m = 0; m < k; ++m) {
      const int ns = (int)peers[m].size();
      for (int i = 0; i < ns; ++i) sets[m].p[i] = reinterpret_cast<const u32x4*>(src[peers[m][i]]->p);
      // members sharing a device split its CUs, so the self-test does not oversubscribe one GPU
      int share = 0;
      for (int d : devs) share += (d == devs[m]);
      const int per = std::max(1, num_cus(devs[m]) * std::max(1, blocks_per_cu) / (ns * share));
      grid[m] = per * ns;
      DeviceGuard g(devs[m]);
      HIP_CHECK(hipStreamCreateWithFlags(&st[m], hipStreamNonBlocking));
      HIP_CHECK(hipEventCreate(&e0[m]));
      HIP_CHECK(hipEventCreate(&e1[m]));
    }
    auto launch_round = [&]() {
      for (int m = 0; m < k; ++m) {
        DeviceGuard g(devs[m]);
        hipLaunchKernelGGL(gather_lds_kernel, dim3(grid[m]), dim3(kBlock), 0, st[m], sets[m], (int)peers[m].size(),
                           (u32x4*)inbox[m]->p, bytes / 16);
        HIP_CHECK(hipGetLastError());
      }
    };
    auto sync_all = [&]() {
      for (int m = 0; m < k; ++m) {
        DeviceGuard g(devs[m]);
        HIP_CHECK(hipStreamSynchronize(st[m]));
      }
    };
    for (int i = 0; i < warmup; ++i) launch_round();
    sync_all();
    auto t0 = std::chrono::steady_clock::now();
    for (int m = 0; m < k; ++m) {
      DeviceGuard g(devs[m]);
      HIP_CHECK(hipEventRecord(e0[m], st[m]));
    }
    for (int i = 0; i < iters; ++i) launch_round();
    for (int m = 0; m < k; ++m) {
      DeviceGuard g(devs[m]);
      HIP_CHECK(hipEventRecord(e1[m], st[m]));
    }
    sync_all();
    wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int m = 0; m < k; ++m) {
      DeviceGuard g(devs[m]);
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, e0[m], e1[m]));
      ms_member[m] = ms;
      (void)hipEventDestroy(e0[m]);
      (void)hipEventDestroy(e1[m]);
      (void)hipStreamDestroy(st[m]);
    }
    // every inbox segment holds its peer's pattern (head and tail windows)
    const size_t words = bytes / 4, win = std::min<size_t>(words, 1 << 14);
    std::vector<unsigned int> h(win);
    for (int m = 0; m < k && ok; ++m) {
      DeviceGuard g(devs[m]);
      for (size_t i = 0; i < peers[m].size() && ok; ++i) {
        const unsigned int seed = seed_of(peers[m][i]);
        for (size_t st0 : {(size_t)0, words - win}) {
          HIP_CHECK(hipMemcpy(h.data(), (const unsigned int*)inbox[m]->p + i * words + st0, win * 4, hipMemcpyDeviceToHost));
          for (size_t w = 0; w < win; ++w)
            if (h[w] != ((unsigned int)((st0 + w) * 2654435761u) ^ seed)) {
              ok = false;
              break;
            }
        }
      }
    }
  }
  py::dict r;
  std::vector<double> gbps(k);
  double bound = 0.0;
  for (int m = 0; m < k; ++m) {
    gbps[m] = (double)bytes * peers[m].size() * iters / (ms_member[m] / 1e3) / 1e9;
    bound = (m == 0) ? gbps[m] : std::min(bound, gbps[m]);
  }
  r["devs"] = devs;
  r["peers"] = peers;
  r["bytes_per_peer"] = bytes;
  r["iters"] = iters;
  r["ms_member"] = ms_member;
  r["wall_ms"] = wall_ms;
  r["ingress_gbps"] = gbps;
  r["bound_gbps"] = bound;
  r["ok"] = ok;
  return r;
}

py::dict to_dict(const CopyResult& c) {
  py::dict r;
  r["src"] = c.src;
  r["dst"] = c.dst;
  r["exec"] = c.exec;
  r["bytes"] = c.bytes;
  r["iters"] = c.iters;
  r["kind"] = c.kind;
  r["nontemporal"] = c.nontemporal;
  r["grid"] = c.grid;
  r["ms_per_iter"] = c.ms_per_iter;
  r["gbps"] = c.gbps;
  r["ok"] = c.ok;
  return r;
}

py::dict copy_bw(int src_dev, int dst_dev, int exec_dev, size_t bytes, int iters, int warmup, const std::string& kind,
                 bool nontemporal, int blocks_per_cu) {
  CopyResult c;
  {
    py::gil_scoped_release nogil;
    c = copy_bw_impl(src_dev, dst_dev, exec_dev, bytes, iters, warmup, kind, nontemporal, blocks_per_cu);
  }
  return to_dict(c);
}

py::dict mfma_warmup(int dev, double target_ms, int iters_per_launch, bool random_operands) {
  py::gil_scoped_release nogil_outer;
  DeviceGuard g(dev);
  if (iters_per_launch < 2 || iters_per_launch % 2) throw std::invalid_argument("iters_per_launch: a positive even number");
  auto* kern = random_operands ? mfma_warmup_random_kernel : mfma_warmup_kernel;
  const int grid = num_cus(dev) * 4;  // 16 waves per CU = 4 per SIMD
  DevBuf out(dev, (size_t)grid * kBlock * sizeof(float));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  int launches = 0;
  float total_ms = 0.f;
  auto t0 = std::chrono::steady_clock::now();
  HIP_CHECK(hipEventRecord(e0, 0));
  do {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, 0, (float*)out.p, iters_per_launch);
    HIP_CHECK(hipGetLastError());
    ++launches;
    HIP_CHECK(hipDeviceSynchronize());
    total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  } while (total_ms < target_ms && launches < 100000);
  // timed launch, clocks now lifted
  HIP_CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, 0, (float*)out.p, iters_per_launch);
  HIP_CHECK(hipEventRecord(e1, 0));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  const double flops = 2.0 * 32 * 32 * 16 * 4.0 * (double)iters_per_launch * (grid * (kBlock / 64));
  py::gil_scoped_acquire gil;
  py::dict r;
  r["device"] = dev;
  r["launches"] = launches;
  r["warm_ms"] = total_ms;
  r["timed_ms"] = ms;
  r["tflops"] = flops / (ms / 1e3) / 1e12;
  r["random_operands"] = random_operands;
  return r;
}

py::dict device_props(int dev) {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, dev));
  char bus[64] = {0};
  HIP_CHECK(hipDeviceGetPCIBusId(bus, sizeof(bus), dev));
  py::dict r;
  r["index"] = dev;
  r["name"] = std::string(p.name);
  r["gcn_arch"] = std::string(p.gcnArchName);
  r["cus"] = p.multiProcessorCount;
  r["total_mem"] = (size_t)p.totalGlobalMem;
  r["lds_per_block"] = (size_t)p.sharedMemPerBlock;
  r["clock_khz"] = p.clockRate;
  r["mem_clock_khz"] = p.memoryClockRate;
  r["mem_bus_width"] = p.memoryBusWidth;
  r["l2_bytes"] = p.l2CacheSize;
  r["pci_bus_id"] = std::string(bus);
  r["warp_size"] = p.warpSize;
  return r;
}

int device_count() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

bool can_access_peer(int a, int b) {
  if (a == b) return true;
  int can = 0;
  HIP_CHECK(hipDeviceCanAccessPeer(&can, a, b));
  return can != 0;
}

// Full ordered-pair matrix: entry [i][j] = GB/s of moving data from device i to device j.
// "read" executes on j (pull over the link), "write" on i (push).  Diagonal = local HBM copy.
std::vector<std::vector<double>> probe_matrix(const std::vector<int>& devs, size_t bytes, int iters, int warmup,
                                              const std::string& mode, const std::string& kind, bool nontemporal,
                                              int blocks_per_cu) {
  const size_t n = devs.size();
  std::vector<std::vector<double>> m(n, std::vector<double>(n, 0.0));
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      int s = devs[i], d = devs[j];
      int ex = (mode == "write") ? s : d;
      CopyResult r = copy_bw_impl(s, d, ex, bytes, iters, warmup, kind, nontemporal, blocks_per_cu);
      if (!r.ok)
        throw std::runtime_error("probe copy verification failed for pair " + std::to_string(s) + "->" + std::to_string(d));
      m[i][j] = r.gbps;
    }
  return m;
}

// XCDs the workgroups of one census launch ran on (on the null stream: the process's own CU mask,
// e.g. HSA_CU_MASK), as {xcc: workgroups}.
py::dict xcc_census(int dev, int blocks) {
  std::vector<unsigned int> host(blocks);
  {
    py::gil_scoped_release nogil;
    DeviceGuard g(dev);
    DevBuf out(dev, (size_t)blocks * sizeof(unsigned int));
    hipLaunchKernelGGL(xcc_census_kernel, dim3(blocks), dim3(64), 0, 0, (unsigned int*)out.p);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpy(host.data(), out.p, (size_t)blocks * sizeof(unsigned int), hipMemcpyDeviceToHost));
  }
  py::dict r;
  for (unsigned int w : host) {
    py::int_ k((int)(w >> 16));
    r[k] = (r.contains(k) ? r[k].cast<int>() : 0) + 1;
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// Cross-process reads through HIP IPC: the mapping RCCL's P2P transport gives a rank of its peers'
// buffers (hipIpcGetMemHandle in the owner, hipIpcOpenMemHandle in the reader).  One process
// exports a patterned buffer; another opens the handle and streams it into a buffer of its own with
// the K1 LDS-DMA kernel, then verifies the pattern.  On one GPU both sides share the device, which
// runs the IPC export / import path (the HSA_ENABLE_IPC_MODE_LEGACY=0 dma-buf handles) and the
// kernel on an imported mapping; on a node the reader is a peer GPU.
class IpcBuffer {
 public:
  IpcBuffer(int dev, size_t bytes, unsigned int seed) : buf_(dev, bytes), seed_(seed) {
    if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
    DeviceGuard g(dev);
    hipLaunchKernelGGL(fill_pattern_kernel, dim3(num_cus(dev) * 4), dim3(kBlock), 0, 0, (unsigned int*)buf_.p, bytes / 4, seed);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipIpcGetMemHandle(&h_, buf_.p));
  }
  py::bytes handle() const { return py::bytes(reinterpret_cast<const char*>(&h_), sizeof(h_)); }
  size_t bytes() const { return buf_.bytes; }
  unsigned int seed() const { return seed_; }
  // After a peer wrote into this buffer through its mapping (K2 over IPC): does it hold pattern(seed)?
  bool holds(unsigned int seed) const {
    py::gil_scoped_release nogil;
    return verify_pattern(buf_, buf_.bytes / 4, seed);
  }

 private:
  DevBuf buf_;
  unsigned int seed_;
  hipIpcMemHandle_t h_{};
};

// Opens another process's buffers by handle for the lifetime of the object.
struct IpcMappings {
  std::vector<void*> p;
  IpcMappings(const std::vector<py::bytes>& handles, int dev) {
    DeviceGuard g(dev);
    for (const py::bytes& hb : handles) {
      const std::string raw = hb;
      if (raw.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("not a hipIpcMemHandle_t");
      hipIpcMemHandle_t h;
      std::memcpy(&h, raw.data(), sizeof(h));
      void* q = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
      p.push_back(q);
    }
  }
  ~IpcMappings() {
    for (void* q : p) (void)hipIpcCloseMemHandle(q);
  }
  IpcMappings(const IpcMappings&) = delete;
  IpcMappings& operator=(const IpcMappings&) = delete;
};

// Event-timed `iters` launches of `launch` on a fresh non-blocking stream (after `warmup` untimed).
template <class F>
float time_launches(F launch, int iters, int warmup) {
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  for (int i = 0; i < warmup; ++i) launch(s);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) launch(s);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(e1, s));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  return ms;
}

// K2 over IPC: the writer's kernel pushes a local patterned buffer into another process's buffer
// through the imported mapping (remote stores, the direction RCCL's P2P write protocol uses).  The
// owner checks the result (IpcBuffer.holds), since only it knows the write has landed in its memory.
py::dict ipc_write_bw(const py::bytes& handle, int dev, size_t bytes, unsigned int seed, int iters, int warmup,
                      int blocks_per_cu) {
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  IpcMappings map({handle}, dev);
  float ms = 0.f;
  {
    py::gil_scoped_release nogil;
    DeviceGuard g(dev);
    DevBuf src(dev, bytes);
    hipLaunchKernelGGL(fill_pattern_kernel, dim3(num_cus(dev) * 4), dim3(kBlock), 0, 0, (unsigned int*)src.p, bytes / 4, seed);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
    const int grid = num_cus(dev) * std::max(1, blocks_per_cu);
    ms = time_launches([&](hipStream_t s) { launch_copy("lds", true, src.p, map.p[0], bytes / 16, grid, s); }, iters, warmup);
  }
  py::dict d;
  d["dev"] = dev;
  d["bytes"] = bytes;
  d["iters"] = iters;
  d["ms_per_iter"] = ms / iters;
  d["gbps"] = (double)bytes / (ms / 1e3 / iters) / 1e9;
  return d;
}

// K5 over IPC: one gather launch pulls every imported buffer at once (segment i of the inbox from
// handle i, as a rank's ingress from all of its peers); each segment is verified against seeds[i].
py::dict ipc_gather_bw(const std::vector<py::bytes>& handles, int dev, size_t bytes, const std::vector<unsigned int>& seeds,
                       int iters, int warmup, int blocks_per_cu) {
  const int nsrc = (int)handles.size();
  if (nsrc < 1 || nsrc > kMaxSrc) throw std::invalid_argument("1..16 handles");
  if (seeds.size() != handles.size()) throw std::invalid_argument("one seed per handle");
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  IpcMappings map(handles, dev);
  float ms = 0.f;
  bool ok = true;
  {
    py::gil_scoped_release nogil;
    DeviceGuard g(dev);
    SrcSet set{};
    for (int i = 0; i < nsrc; ++i) set.p[i] = reinterpret_cast<const u32x4*>(map.p[i]);
    DevBuf inbox(dev, bytes * (size_t)nsrc);
    const int per = std::max(1, num_cus(dev) * std::max(1, blocks_per_cu) / nsrc);
    const int grid = per * nsrc;  // every source gets the same block count
    ms = time_launches([&](hipStream_t s) {
      hipLaunchKernelGGL(gather_lds_kernel, dim3(grid), dim3(kBlock), 0, s, set, nsrc, (u32x4*)inbox.p, bytes / 16);
    }, iters, warmup);
    const size_t words = bytes / 4, win = std::min<size_t>(words, 1 << 14);
    std::vector<unsigned int> h(win);
    for (int i = 0; i < nsrc && ok; ++i)
      for (size_t st0 : {(size_t)0, words / 2 - std::min(words / 2, win / 2), words - win}) {
        HIP_CHECK(hipMemcpy(h.data(), (const unsigned int*)inbox.p + (size_t)i * words + st0, win * 4, hipMemcpyDeviceToHost));
        for (size_t w = 0; w < win; ++w)
          if (h[w] != ((unsigned int)((st0 + w) * 2654435761u) ^ seeds[i])) {
            ok = false;
            break;
          }
      }
  }
  py::dict d;
  d["dev"] = dev;
  d["segments"] = nsrc;
  d["bytes_per_segment"] = bytes;
  d["iters"] = iters;
  d["ms_per_iter"] = ms / iters;
  d["gbps"] = (double)bytes * nsrc / (ms / 1e3 / iters) / 1e9;
  d["ok"] = ok;
  return d;
}

py::dict ipc_read_bw(const py::bytes& handle, int dev, size_t bytes, unsigned int seed, int iters, int warmup,
                     int blocks_per_cu) {
  const std::string raw = handle;
  if (raw.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("not a hipIpcMemHandle_t");
  if (bytes < 16 || bytes % 16) throw std::invalid_argument("bytes must be a positive multiple of 16");
  if (iters < 1) throw std::invalid_argument("iters >= 1");
  hipIpcMemHandle_t h;
  std::memcpy(&h, raw.data(), sizeof(h));
  DeviceGuard g(dev);
  void* src = nullptr;
  HIP_CHECK(hipIpcOpenMemHandle(&src, h, hipIpcMemLazyEnablePeerAccess));
  struct Closer {
    void* p;
    ~Closer() { (void)hipIpcCloseMemHandle(p); }
  } closer{src};
  DevBuf dst(dev, bytes);
  const size_t n_vec = bytes / 16;
  const int grid = num_cus(dev) * std::max(1, blocks_per_cu);
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  for (int i = 0; i < warmup; ++i) launch_copy("lds", true, src, dst.p, n_vec, grid, s);
  HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) launch_copy("lds", true, src, dst.p, n_vec, grid, s);
  HIP_CHECK(hipEventRecord(e1, s));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  HIP_CHECK(hipStreamDestroy(s));
  const bool ok = verify_pattern(dst, bytes / 4, seed);
  py::dict d;
  d["dev"] = dev;
  d["bytes"] = bytes;
  d["iters"] = iters;
  d["ms_per_iter"] = ms / iters;
  d["gbps"] = (double)bytes / (ms / 1e3 / iters) / 1e9;
  d["ok"] = ok;
  return d;
}

}  // namespace

PYBIND11_MODULE(_probe, m) {
  m.doc() = "HIP/CDNA4 (gfx950) link probe kernels: LDS-DMA staged p2p/HBM copy, MFMA warm-up";
  m.def("device_count", &device_count);
  m.def("device_props", &device_props, py::arg("dev"));
  m.def("can_access_peer", &can_access_peer, py::arg("a"), py::arg("b"));
  m.def("copy_bw", &copy_bw, py::arg("src_dev"), py::arg("dst_dev"), py::arg("exec_dev"), py::arg("bytes"),
        py::arg("iters") = 10, py::arg("warmup") = 2, py::arg("kind") = "lds", py::arg("nontemporal") = false,
        py::arg("blocks_per_cu") = kBlocksPerCU);
  m.def("gather_bw", &gather_bw, py::arg("dst_dev"), py::arg("srcs"), py::arg("bytes") = (size_t)64 << 20,
        py::arg("iters") = 3, py::arg("warmup") = 1, py::arg("blocks_per_cu") = kBlocksPerCU);
  m.def("ring_bw", &ring_bw, py::arg("devs"), py::arg("peers"), py::arg("bytes") = (size_t)64 << 20, py::arg("iters") = 3,
        py::arg("warmup") = 1, py::arg("blocks_per_cu") = kBlocksPerCU);
  m.def("mfma_warmup", &mfma_warmup, py::arg("dev"), py::arg("target_ms") = 50.0, py::arg("iters_per_launch") = 4096,
        py::arg("random_operands") = false);
  m.def("probe_matrix", &probe_matrix, py::arg("devs"), py::arg("bytes") = (size_t)256 << 20, py::arg("iters") = 5,
        py::arg("warmup") = 1, py::arg("mode") = "read", py::arg("kind") = "lds", py::arg("nontemporal") = false,
        py::arg("blocks_per_cu") = kBlocksPerCU, py::call_guard<py::gil_scoped_release>());
  m.def("xcc_census", &xcc_census, py::arg("dev"), py::arg("blocks") = 4096);
  py::class_<IpcBuffer>(m, "IpcBuffer")
      .def(py::init<int, size_t, unsigned int>(), py::arg("dev"), py::arg("bytes"), py::arg("seed") = 0x5eedu)
      .def("handle", &IpcBuffer::handle)
      .def("holds", &IpcBuffer::holds, py::arg("seed"), "does the buffer hold pattern(seed)? (after a peer's IPC write)")
      .def_property_readonly("bytes", &IpcBuffer::bytes)
      .def_property_readonly("seed", &IpcBuffer::seed);
  m.def("ipc_write_bw", &ipc_write_bw, py::arg("handle"), py::arg("dev"), py::arg("bytes"), py::arg("seed"),
        py::arg("iters") = 5, py::arg("warmup") = 1, py::arg("blocks_per_cu") = kBlocksPerCU,
        "K2 over IPC: push pattern(seed) into another process's buffer through its handle (owner verifies)");
  m.def("ipc_gather_bw", &ipc_gather_bw, py::arg("handles"), py::arg("dev"), py::arg("bytes"), py::arg("seeds"),
        py::arg("iters") = 5, py::arg("warmup") = 1, py::arg("blocks_per_cu") = kBlocksPerCU,
        "K5 over IPC: one gather launch over every imported buffer; each segment verified");
  m.def("ipc_read_bw", &ipc_read_bw, py::arg("handle"), py::arg("dev"), py::arg("bytes"), py::arg("seed"),
        py::arg("iters") = 5, py::arg("warmup") = 1, py::arg("blocks_per_cu") = kBlocksPerCU,
        "open another process's buffer by its IPC handle and stream it into a local one (K1 kernel); verified");
  m.attr("BLOCK") = kBlock;
  m.attr("UNROLL") = kUnroll;
  m.attr("BLOCKS_PER_CU") = kBlocksPerCU;
}
