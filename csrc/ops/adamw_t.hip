// AdamW that also writes the transposed bf16 weights.
//
// The Llama workload's backward GEMMs run in hipBLASLt's fastest ("NT") layout, whose input-gradient
// GEMM reads W^T (models/llama.py).  W changes only in the optimizer step, yet round 3 re-made every
// W^T in every backward: 16 GB read + 16 GB written per step by the transpose kernel.  Here the
// optimizer, which streams every weight anyway (master/m/v/grad in, master/m/v/W out), writes W^T in
// the same pass: +2 B per element on top of its 28 B, and the backward finds W^T ready.
//
//   adamw_tiles_kernel   one 64 x 256 tile of one projection matrix per loop trip (grid-stride over
//                        every matrix's tiles: the persistent grid ends when the tile index passes the
//                        total, so every wave exits).  The update walks 1 KiB row segments like the
//                        flat kernel, stages the new bf16 rows in an XOR-swizzled LDS tile, and writes
//                        8 consecutive rows of one column of W^T per 16-B store (conflict-free).
//   adamw_ranges_kernel  the parameters that are not transposed (embedding, norms): blockIdx.y picks a
//                        range, grid-stride over its 16-B vectors.
// Both apply exactly adamw_body's arithmetic (csrc/ops/fused_ops.hip), in the same per-element order,
// so the master/m/v/W bits equal the flat kernel's.  DEV = the graph-capturable form: bias
// corrections and the clipping factor are derived on the device (adamw_dev_kernel's contract).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>
#include <vector>

namespace gtk_adamw {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

struct Hyper {
  float lr, b1, b2, eps, wd, gs, bc1, bc2;
};

// hp (host form)  = [lr, b1, b2, eps, wd, grad_scale, bias_c1, bias_c2]
// hp (DEV form)   = [lr, b1, b2, eps, wd, grad_scale, clip_norm (<= 0: off), -], + partials + step count
template <bool DEV>
__device__ __forceinline__ Hyper hyper(const float* __restrict__ hp, const float* __restrict__ part, int nparts,
                                       const float* __restrict__ tptr) {
  Hyper h{hp[0], hp[1], hp[2], hp[3], hp[4], hp[5], 0.f, 0.f};
  if (!DEV) {
    h.bc1 = hp[6];
    h.bc2 = hp[7];
    return h;
  }
  __shared__ float red[4];
  const float clip = hp[6];
  if (nparts > 0 && clip > 0.f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * h.gs;
    h.gs = h.gs * fminf(1.f, clip / (norm + 1e-6f));
  }
  const float t = tptr[0];
  h.bc1 = 1.f - powf(h.b1, t);
  h.bc2 = 1.f - powf(h.b2, t);
  return h;
}

// 8 gradient elements at flat index i: bf16, or fp32 after a DP all-reduce in fp32
__device__ __forceinline__ void load_g8(const u16* __restrict__ g, size_t i, float (&out)[8]) {
  const u16x8 gv = *reinterpret_cast<const u16x8*>(g + i);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bf2f(gv[j]);
}
__device__ __forceinline__ void load_g8(const float* __restrict__ g, size_t i, float (&out)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(g + i), b = *reinterpret_cast<const f32x4*>(g + i + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = a[j], out[j + 4] = b[j];
}

// 8 elements at flat index i (a multiple of 8): the same expressions, in the same order, as
// adamw_body in fused_ops.hip
template <typename G>
__device__ __forceinline__ u16x8 adam8(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                       const G* __restrict__ g, u16* __restrict__ w, size_t i, const Hyper& h) {
  f32x4* mp = reinterpret_cast<f32x4*>(master + i);
  f32x4* mm_ = reinterpret_cast<f32x4*>(m + i);
  f32x4* vp = reinterpret_cast<f32x4*>(v + i);
  f32x4 p0 = mp[0], p1 = mp[1], m0 = mm_[0], m1 = mm_[1], v0 = vp[0], v1 = vp[1];
  float gf[8];
  load_g8(g, i, gf);
  u16x8 wo;
  float p[8], mm[8], vv[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p[j] = p0[j], p[j + 4] = p1[j];
    mm[j] = m0[j], mm[j + 4] = m1[j];
    vv[j] = v0[j], vv[j + 4] = v1[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gr = gf[j] * h.gs;
    mm[j] = h.b1 * mm[j] + (1.f - h.b1) * gr;
    vv[j] = h.b2 * vv[j] + (1.f - h.b2) * gr * gr;
    const float upd = (mm[j] / h.bc1) / (sqrtf(vv[j] / h.bc2) + h.eps);
    p[j] = p[j] - h.lr * (upd + h.wd * p[j]);
    wo[j] = f2bf(p[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p0[j] = p[j], p1[j] = p[j + 4];
    m0[j] = mm[j], m1[j] = mm[j + 4];
    v0[j] = vv[j], v1[j] = vv[j + 4];
  }
  mp[0] = p0, mp[1] = p1, mm_[0] = m0, mm_[1] = m1, vp[0] = v0, vp[1] = v1;
  *reinterpret_cast<u16x8*>(w + i) = wo;
  return wo;
}

// adam8 split in two: the loads of 8 elements, then the update and stores from those registers.
// The tile kernel issues the loads of several passes before any store: through the same master/m/v
// pointers the compiler cannot hoist a later pass's loads above an earlier pass's stores.
struct Adam8In {
  f32x4 p0, p1, m0, m1, v0, v1;
  float gf[8];
};
template <typename G>
__device__ __forceinline__ void adam8_load(const float* __restrict__ master, const float* __restrict__ m, const float* __restrict__ v,
                                           const G* __restrict__ g, size_t i, Adam8In& in) {
  const f32x4* mp = reinterpret_cast<const f32x4*>(master + i);
  const f32x4* mm_ = reinterpret_cast<const f32x4*>(m + i);
  const f32x4* vp = reinterpret_cast<const f32x4*>(v + i);
  in.p0 = mp[0], in.p1 = mp[1], in.m0 = mm_[0], in.m1 = mm_[1], in.v0 = vp[0], in.v1 = vp[1];
  load_g8(g, i, in.gf);
}
__device__ __forceinline__ u16x8 adam8_store(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                             u16* __restrict__ w, size_t i, const Adam8In& in, const Hyper& h) {
  u16x8 wo;
  float p[8], mm[8], vv[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p[j] = in.p0[j], p[j + 4] = in.p1[j];
    mm[j] = in.m0[j], mm[j + 4] = in.m1[j];
    vv[j] = in.v0[j], vv[j + 4] = in.v1[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // adamw_body's expressions, in its order
    const float gr = in.gf[j] * h.gs;
    mm[j] = h.b1 * mm[j] + (1.f - h.b1) * gr;
    vv[j] = h.b2 * vv[j] + (1.f - h.b2) * gr * gr;
    const float upd = (mm[j] / h.bc1) / (sqrtf(vv[j] / h.bc2) + h.eps);
    p[j] = p[j] - h.lr * (upd + h.wd * p[j]);
    wo[j] = f2bf(p[j]);
  }
  f32x4 p0, p1, m0, m1, v0, v1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p0[j] = p[j], p1[j] = p[j + 4];
    m0[j] = mm[j], m1[j] = mm[j + 4];
    v0[j] = vv[j], v1[j] = vv[j + 4];
  }
  f32x4* mp = reinterpret_cast<f32x4*>(master + i);
  f32x4* mmp = reinterpret_cast<f32x4*>(m + i);
  f32x4* vp = reinterpret_cast<f32x4*>(v + i);
  mp[0] = p0, mp[1] = p1, mmp[0] = m0, mmp[1] = m1, vp[0] = v0, vp[1] = v1;
  *reinterpret_cast<u16x8*>(w + i) = wo;
  return wo;
}

// one transposed matrix: rows R x cols C at flat element offset `off`, its W^T ([C, R]) at `toff` of
// the transposed buffer, tiles [tile_base, tile_base + (R/64)(C/64)) of the global tile index
struct Mat {
  int64_t off, toff, R, C, tile_base;
};

// Tile = 64 rows x 256 columns.  The fp32 master/m/v streams are read and written in 1 KiB
// contiguous row segments (a wave covers two rows: 64 lanes x 8 elements x 4 B), the access shape of
// the flat kernel; a 64 x 64 tile's 256-B segments ran the step at 5.45 TB/s against the flat
// kernel's 5.97 (profiles/r04_llama).  W^T leaves as 256 output rows x 128 B.
constexpr int kTR = 64, kTC = 256;

template <bool DEV, typename G, int kAhead = 1>
__global__ __launch_bounds__(256) void adamw_tiles_kernel(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                                          const G* __restrict__ g, u16* __restrict__ w, u16* __restrict__ wt,
                                                          const Mat* __restrict__ mats, int nmats, int64_t total_tiles,
                                                          const float* __restrict__ hp, const float* __restrict__ part, int nparts,
                                                          const float* __restrict__ tptr) {
  // [row][16-B vector]: vector v of row r at slot v ^ ((r >> 3) & 7) -- the XOR touches the low 3 bits
  // only, so a row's 32 vectors stay a permutation of its own 512 B
  __shared__ u16x8 tile[kTR][kTC / 8];
  const Hyper h = hyper<DEV>(hp, part, nparts, tptr);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
  for (int64_t ti = blockIdx.x; ti < total_tiles; ti += gridDim.x) {
    int lo = 0, hi = nmats - 1;  // last matrix whose tile_base <= ti (block-uniform)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (mats[mid].tile_base <= ti) lo = mid;
      else hi = mid - 1;
    }
    const Mat mt = mats[lo];
    const int64_t local = ti - mt.tile_base, tiles_c = mt.C / kTC;
    const int64_t r0 = (local / tiles_c) * kTR, c0 = (local % tiles_c) * kTC;
    // update: 8 passes of 8 rows; thread t takes vector t & 31 of row 8 * pass + t / 32
    if (kAhead == 1) {
#pragma unroll 4
      for (int pass = 0; pass < kTR / 8; ++pass) {
        const int r = 8 * pass + (t >> 5), vv = t & 31;
        const u16x8 wo = adam8(master, m, v, g, w, (size_t)(mt.off + (r0 + r) * mt.C + c0 + 8 * vv), h);
        tile[r][vv ^ ((r >> 3) & 7)] = wo;
      }
    } else {  // kAhead passes' loads in flight before their stores
#pragma unroll 1
      for (int p0 = 0; p0 < kTR / 8; p0 += kAhead) {
        Adam8In in[kAhead];
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
          const int r = 8 * (p0 + u) + (t >> 5), vv = t & 31;
          adam8_load(master, m, v, g, (size_t)(mt.off + (r0 + r) * mt.C + c0 + 8 * vv), in[u]);
        }
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
          const int r = 8 * (p0 + u) + (t >> 5), vv = t & 31;
          tile[r][vv ^ ((r >> 3) & 7)] = adam8_store(master, m, v, w, (size_t)(mt.off + (r0 + r) * mt.C + c0 + 8 * vv), in[u], h);
        }
      }
    }
    __syncthreads();
    // transposed write: per instruction a wave takes one 16-B column vector vc (8 columns) x the 8
    // row groups p, lanes (p, column & 7): the row groups sit on 8 different slots, the 8 columns in
    // one slot's 4 dwords -- 32 banks, no conflicts; each output row gets 8 x 16 B = 128 B
    const int p = lane >> 3, cl = lane & 7;
#pragma unroll 4
    for (int i = 0; i < kTC / 32; ++i) {
      const int vc = 4 * i + wv;
      const int c = 8 * vc + cl;
      const int slot = vc ^ p;
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = lds[((8 * p + j) * (kTC / 8) + slot) * 8 + cl];
      *reinterpret_cast<u16x8*>(wt + mt.toff + (c0 + c) * mt.R + r0 + 8 * p) = o;
    }
    __syncthreads();  // the tile is free for the next trip
  }
}

// ranges: [start, length] element pairs (multiples of 8)
template <bool DEV, typename G>
__global__ __launch_bounds__(256) void adamw_ranges_kernel(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                                           const G* __restrict__ g, u16* __restrict__ w,
                                                           const int64_t* __restrict__ ranges, const float* __restrict__ hp,
                                                           const float* __restrict__ part, int nparts,
                                                           const float* __restrict__ tptr) {
  const Hyper h = hyper<DEV>(hp, part, nparts, tptr);
  const int64_t start = ranges[2 * blockIdx.y], nv = ranges[2 * blockIdx.y + 1] >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256)
    adam8(master, m, v, g, w, (size_t)(start + 8 * i), h);
}

#define CHECK_DEV(t, dt) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == (dt) && (t).is_contiguous(), #t " has the wrong type/device")

template <typename G>
void launch(at::Tensor& master, at::Tensor& m, at::Tensor& v, const G* gp, at::Tensor& w, at::Tensor& wt, const at::Tensor& hp,
            const at::Tensor& mats, int64_t total_tiles, const at::Tensor& ranges, int64_t max_range,
            const c10::optional<at::Tensor>& part, const c10::optional<at::Tensor>& t, int64_t ahead_arg) {
  const bool dev = t.has_value();
  const float* pp = nullptr;
  int np = 0;
  if (part.has_value()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous(), "adamw_step_t: bad part");
    pp = part->data_ptr<float>();
    np = (int)part->numel();
  }
  const float* tp = dev ? t->data_ptr<float>() : nullptr;
  hipStream_t s = at::hip::getCurrentHIPStream().stream();
  auto* mp = master.data_ptr<float>();
  auto* mmp = m.data_ptr<float>();
  auto* vp = v.data_ptr<float>();
  auto* wp = reinterpret_cast<u16*>(w.data_ptr());
  auto* wtp = reinterpret_cast<u16*>(wt.data_ptr());
  if (mats.size(0) > 0 && total_tiles > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>(total_tiles, 4096);
    const Mat* md = reinterpret_cast<const Mat*>(mats.data_ptr<int64_t>());
    const int ahead = ahead_arg == 2 || ahead_arg == 4 ? (int)ahead_arg : 1;  // passes' loads in flight (A/B)
    if (dev)
      hipLaunchKernelGGL((adamw_tiles_kernel<true, G>), dim3(grid), dim3(256), 0, s, mp, mmp, vp, gp, wp, wtp, md, (int)mats.size(0),
                         total_tiles, hp.data_ptr<float>(), pp, np, tp);
    else if (ahead == 4)
      hipLaunchKernelGGL((adamw_tiles_kernel<false, G, 4>), dim3(grid), dim3(256), 0, s, mp, mmp, vp, gp, wp, wtp, md,
                         (int)mats.size(0), total_tiles, hp.data_ptr<float>(), pp, np, tp);
    else if (ahead == 2)
      hipLaunchKernelGGL((adamw_tiles_kernel<false, G, 2>), dim3(grid), dim3(256), 0, s, mp, mmp, vp, gp, wp, wtp, md,
                         (int)mats.size(0), total_tiles, hp.data_ptr<float>(), pp, np, tp);
    else
      hipLaunchKernelGGL((adamw_tiles_kernel<false, G>), dim3(grid), dim3(256), 0, s, mp, mmp, vp, gp, wp, wtp, md,
                         (int)mats.size(0), total_tiles, hp.data_ptr<float>(), pp, np, tp);
  }
  if (ranges.size(0) > 0 && max_range > 0) {
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_range / 8 + 255) / 256, 2048));
    const dim3 grid(gx, (unsigned)ranges.size(0));
    if (dev)
      hipLaunchKernelGGL((adamw_ranges_kernel<true, G>), grid, dim3(256), 0, s, mp, mmp, vp, gp, wp, ranges.data_ptr<int64_t>(),
                         hp.data_ptr<float>(), pp, np, tp);
    else
      hipLaunchKernelGGL((adamw_ranges_kernel<false, G>), grid, dim3(256), 0, s, mp, mmp, vp, gp, wp, ranges.data_ptr<int64_t>(),
                         hp.data_ptr<float>(), pp, np, tp);
  }
}

// mats: int64 [N, 5] (off, toff, R, C, tile_base) on the device; ranges: int64 [M, 2] on the device.
// part / t present = the DEV form (hp in adamw_step_dev's layout).
void adamw_step_t(at::Tensor& master, at::Tensor& m, at::Tensor& v, const at::Tensor& g, at::Tensor& w, at::Tensor& wt,
                  const at::Tensor& hp, const at::Tensor& mats, int64_t total_tiles, const at::Tensor& ranges,
                  int64_t max_range, c10::optional<at::Tensor> part, c10::optional<at::Tensor> t, int64_t ahead) {
  CHECK_DEV(master, at::kFloat);
  CHECK_DEV(m, at::kFloat);
  CHECK_DEV(v, at::kFloat);
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat),
              "adamw_step_t: g must be a contiguous bf16 or fp32 GPU tensor");
  CHECK_DEV(w, at::kBFloat16);
  CHECK_DEV(wt, at::kBFloat16);
  CHECK_DEV(hp, at::kFloat);
  CHECK_DEV(mats, at::kLong);
  CHECK_DEV(ranges, at::kLong);
  const int64_t n = master.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n && w.numel() == n, "adamw_step_t: flat buffers differ in size");
  TORCH_CHECK(mats.dim() == 2 && mats.size(1) == 5 && ranges.dim() == 2 && ranges.size(1) == 2, "adamw_step_t: bad descriptors");
  TORCH_CHECK(ranges.size(0) <= 65535, "adamw_step_t: too many ranges");
  if (g.scalar_type() == at::kFloat)
    launch(master, m, v, g.data_ptr<float>(), w, wt, hp, mats, total_tiles, ranges, max_range, part, t, ahead);
  else
    launch(master, m, v, reinterpret_cast<const u16*>(g.data_ptr()), w, wt, hp, mats, total_tiles, ranges, max_range, part, t,
           ahead);
}

}  // namespace gtk_adamw
