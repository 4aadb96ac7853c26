// Fused elementwise / normalisation / loss / optimizer kernels for the Llama-3 DP validation
// workload (BASELINE config 5: "Llama-3-8B DP all-reduce training on the allocated set").
//
// The reference has no model code; these kernels exist because the validation
// workload's non-GEMM ops are HBM-bound and a bf16 Llama step on MI355X would otherwise spend its
// time in chains of small PyTorch elementwise kernels.  GEMMs stay on hipBLASLt (plain library
// GEMMs); everything between them is one pass over HBM here:
//   rmsnorm_fwd / rmsnorm_bwd   wave-per-row, 16-B vector loads, no LDS (D=4096 -> 8 x 16 B per lane),
//                               bwd keeps per-lane dW partials in registers across rows
//   rope_split_fwd / _bwd       QKV GEMM output [T, (H+2Hkv)*Dh] -> q/k/v in [B, heads, S, Dh] with
//                               RoPE applied to q,k in the same pass (and the exact inverse)
//   swiglu_fwd / swiglu_bwd     gate|up GEMM output [T, 2F] -> silu(g)*u, and its gradient
//   xent_fwd / xent_bwd         fused log-softmax cross-entropy over V=128256, gradient written
//                               in place over the bf16 logits (saves a T x V fp32 tensor)
//   adamw_step / sq_norm        one flat-buffer AdamW over bf16 params + fp32 master/m/v, and the
//                               global gradient-norm reduction for clipping
//   adamw_step_dev /            the graph-capturable pair: step count, bias corrections and the
//   sq_norm_parts               clipping factor live on the device (2 launches per optimizer step)
//   mnist_synth                 the MNIST workload's synthetic batch, one launch, device-indexed
// All math in fp32, bf16 storage.  Wave size 64 everywhere (gfx950).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>

namespace {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

#define CHECK_BF16(t) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == at::kBFloat16 && (t).is_contiguous(), #t " must be a contiguous bf16 GPU tensor")
#define CHECK_GRAD(t) TORCH_CHECK((t).is_cuda() && ((t).scalar_type() == at::kBFloat16 || (t).scalar_type() == at::kFloat) && (t).is_contiguous(), #t " must be a contiguous bf16 or fp32 GPU tensor")
#define CHECK_F32(t) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == at::kFloat && (t).is_contiguous(), #t " must be a contiguous fp32 GPU tensor")

const u16* bp(const at::Tensor& t) { return reinterpret_cast<const u16*>(t.data_ptr()); }
u16* bpm(at::Tensor& t) { return reinterpret_cast<u16*>(t.data_ptr()); }

// =============================================================================== RMSNorm
// One wave per row; lane l owns vectors c = i*64 + l (8 bf16 each).  NV = ceil(D / 512).
// ADD: h = bf16(x + res) is formed in registers, written once (the residual stream) and normalised
// in the same pass — the separate add kernel and its re-read of h disappear.
template <int NV, bool ADD = false>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ w,
                                                          u16* __restrict__ y, float* __restrict__ rstd, int M, int D,
                                                          float eps, const u16* __restrict__ res = nullptr,
                                                          u16* __restrict__ h = nullptr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nvec = D >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)row * D);
  u16x8 v[NV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 64 + lane;
    if (c < nvec) {
      v[i] = xr[c];
      if constexpr (ADD) {
        const u16x8 rv = reinterpret_cast<const u16x8*>(res + (size_t)row * D)[c];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = f2bf(bf2f(v[i][j]) + bf2f(rv[j]));
        reinterpret_cast<u16x8*>(h + (size_t)row * D)[c] = v[i];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = bf2f(v[i][j]);
        ss += f * f;
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0) rstd[row] = r;
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8* yr = reinterpret_cast<u16x8*>(y + (size_t)row * D);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 64 + lane;
    if (c < nvec) {
      u16x8 wv = wr[c], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[i][j]) * r * bf2f(wv[j]));
      yr[c] = o;
    }
  }
}

// dx = r*g - x*r^3*mean(g*x), g = dy*w ;  dW partial[wave] = sum_rows dy*x*r  (fp32, reduced later)
// ACC: dx += dres (the residual stream's own gradient) before the single bf16 rounding — replaces
// autograd's separate accumulate kernel for the fused add+norm.
template <int NV, bool ACC = false>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                          const u16* __restrict__ w, const float* __restrict__ rstd,
                                                          u16* __restrict__ dx, float* __restrict__ dw_part, int M, int D,
                                                          const u16* __restrict__ dres = nullptr) {
  const int lane = threadIdx.x & 63;
  const int gwave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int nvec = D >> 3;
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  float dwacc[NV][8];
  u16x8 wv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 64 + lane;
    if (c < nvec) wv[i] = wr[c];
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
  }
  // one wave per SIMD walks its rows with the NEXT row's x / dy / dres loads in flight while it
  // computes the current one (the grid is one wave per SIMD, so the second register set is free):
  // at one outstanding row per wave the kernel was latency-bound at 4.2 TB/s (profiles/r04_norm)
  u16x8 xv[NV], gv[NV], dv[ACC ? NV : 1];
  u16x8 nx[NV], ng[NV], nd[ACC ? NV : 1];
  auto load_row = [&](int row, u16x8 (&a)[NV], u16x8 (&b)[NV], u16x8 (&cc)[ACC ? NV : 1]) {
    const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)row * D);
    const u16x8* dyr = reinterpret_cast<const u16x8*>(dy + (size_t)row * D);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 64 + lane;
      if (c < nvec) {
        a[i] = xr[c];
        b[i] = dyr[c];
        if constexpr (ACC) cc[i] = reinterpret_cast<const u16x8*>(dres + (size_t)row * D)[c];
      }
    }
  };
  if (gwave < M) load_row(gwave, xv, gv, dv);
  for (int row = gwave; row < M; row += nwaves) {
    const float r = rstd[row];
    if (row + nwaves < M) load_row(row + nwaves, nx, ng, nd);
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 64 + lane;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = bf2f(xv[i][j]), dyf = bf2f(gv[i][j]);
          dot += dyf * bf2f(wv[i][j]) * xf;
          dwacc[i][j] += dyf * xf * r;
        }
      }
    }
    dot = wave_sum(dot);
    const float k = r * r * r * dot / (float)D;
    u16x8* dxr = reinterpret_cast<u16x8*>(dx + (size_t)row * D);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 64 + lane;
      if (c < nvec) {
        u16x8 o;
        if constexpr (ACC) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            o[j] = f2bf(r * bf2f(gv[i][j]) * bf2f(wv[i][j]) - bf2f(xv[i][j]) * k + bf2f(dv[i][j]));
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(r * bf2f(gv[i][j]) * bf2f(wv[i][j]) - bf2f(xv[i][j]) * k);
        }
        dxr[c] = o;
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      xv[i] = nx[i];
      gv[i] = ng[i];
      if constexpr (ACC) dv[i] = nd[i];
    }
  }
  float* part = dw_part + (size_t)gwave * D;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 64 + lane;
    if (c < nvec) {
      f32x4 a = {dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]};
      f32x4 b = {dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]};
      reinterpret_cast<f32x4*>(part)[2 * c] = a;
      reinterpret_cast<f32x4*>(part)[2 * c + 1] = b;
    }
  }
}

// dW = column sums of the [P, D] fp32 partials, written as bf16 in one launch.  Each block owns 16
// columns so that D = 4096 gives 256 blocks, one per CU; a wave-instruction reads 4 rows x 64 B.  The
// 64 row streams of a block (16 waves x 4 lane groups) combine through LDS in a fixed order: no
// atomics, so dW is bitwise reproducible run to run.
constexpr int kColWaves = 16, kColW = 16;
__global__ __launch_bounds__(64 * kColWaves) void colsum_bf16_kernel(const float* __restrict__ part, u16* __restrict__ dw,
                                                                     int P, int D) {
  constexpr int kStreams = kColWaves * (64 / kColW);
  __shared__ float red[kStreams][kColW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane % kColW, stream = wave * (64 / kColW) + lane / kColW;
  const int col = blockIdx.x * kColW + c;
  float s = 0.f;
  if (col < D)
    for (int p = stream; p < P; p += kStreams) s += part[(size_t)p * D + col];
  red[stream][c] = s;
  __syncthreads();
  if (threadIdx.x < kColW && col < D) {
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < kStreams; ++i) t += red[i][c];
    dw[col] = f2bf(t);
  }
}

template <int NV>
void rmsnorm_fwd_launch(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, at::Tensor& rstd, int M, int D, float eps) {
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<NV>, dim3((M + 3) / 4), dim3(256), 0, cur_stream(), bp(x), bp(w), bpm(y),
                     rstd.data_ptr<float>(), M, D, eps);
}

template <int NV>
void add_rmsnorm_fwd_launch(const at::Tensor& x, const at::Tensor& r, const at::Tensor& w, at::Tensor& h, at::Tensor& y,
                            at::Tensor& rstd, int M, int D, float eps) {
  hipLaunchKernelGGL((rmsnorm_fwd_kernel<NV, true>), dim3((M + 3) / 4), dim3(256), 0, cur_stream(), bp(x), bp(w), bpm(y),
                     rstd.data_ptr<float>(), M, D, eps, bp(r), bpm(h));
}

// h = x + r (bf16), y = rmsnorm(h) * w in one pass; returns {h, y, rstd}.
std::vector<at::Tensor> add_rmsnorm_fwd(const at::Tensor& x, const at::Tensor& r, const at::Tensor& w, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(r);
  CHECK_BF16(w);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192 && w.numel() == D, "add_rmsnorm: D must be a multiple of 8, <= 8192, and match w");
  TORCH_CHECK(r.sizes() == x.sizes(), "add_rmsnorm: x and r shapes differ");
  const int M = (int)(x.numel() / D);
  auto h = at::empty_like(x);
  auto y = at::empty_like(x);
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  if (M == 0) return {h, y, rstd};
  const int nv = (D + 511) / 512;
  if (nv <= 1) add_rmsnorm_fwd_launch<1>(x, r, w, h, y, rstd, M, D, (float)eps);
  else if (nv <= 2) add_rmsnorm_fwd_launch<2>(x, r, w, h, y, rstd, M, D, (float)eps);
  else if (nv <= 4) add_rmsnorm_fwd_launch<4>(x, r, w, h, y, rstd, M, D, (float)eps);
  else if (nv <= 8) add_rmsnorm_fwd_launch<8>(x, r, w, h, y, rstd, M, D, (float)eps);
  else add_rmsnorm_fwd_launch<16>(x, r, w, h, y, rstd, M, D, (float)eps);
  return {h, y, rstd};
}

std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192 && w.numel() == D, "rmsnorm: D must be a multiple of 8, <= 8192, and match w");
  const int M = (int)(x.numel() / D);
  auto y = at::empty_like(x);
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  if (M == 0) return {y, rstd};
  const int nv = (D + 511) / 512;
  if (nv <= 1) rmsnorm_fwd_launch<1>(x, w, y, rstd, M, D, (float)eps);
  else if (nv <= 2) rmsnorm_fwd_launch<2>(x, w, y, rstd, M, D, (float)eps);
  else if (nv <= 4) rmsnorm_fwd_launch<4>(x, w, y, rstd, M, D, (float)eps);
  else if (nv <= 8) rmsnorm_fwd_launch<8>(x, w, y, rstd, M, D, (float)eps);
  else rmsnorm_fwd_launch<16>(x, w, y, rstd, M, D, (float)eps);
  return {y, rstd};
}

template <int NV>
void rmsnorm_bwd_launch(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd, at::Tensor& dx,
                        at::Tensor& part, int grid, int M, int D, const u16* dres) {
  if (dres)
    hipLaunchKernelGGL((rmsnorm_bwd_kernel<NV, true>), dim3(grid), dim3(256), 0, cur_stream(), bp(dy), bp(x), bp(w),
                       rstd.data_ptr<float>(), bpm(dx), part.data_ptr<float>(), M, D, dres);
  else
    hipLaunchKernelGGL((rmsnorm_bwd_kernel<NV, false>), dim3(grid), dim3(256), 0, cur_stream(), bp(dy), bp(x), bp(w),
                       rstd.data_ptr<float>(), bpm(dx), part.data_ptr<float>(), M, D, nullptr);
}

std::vector<at::Tensor> rmsnorm_bwd_impl(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd,
                                         const u16* dres, const at::Tensor* dw_out = nullptr);

std::vector<at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd) {
  return rmsnorm_bwd_impl(dy, x, w, rstd, nullptr);
}

// the same, with dW written into `dw_out` (a contiguous bf16 view of D elements, e.g. the weight's
// slot of the flat gradient buffer): no separate dW tensor for autograd to accumulate
at::Tensor rmsnorm_bwd_into(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd,
                            const at::Tensor& dw_out) {
  return rmsnorm_bwd_impl(dy, x, w, rstd, nullptr, &dw_out)[0];
}

// Backward of add_rmsnorm: dx = rmsnorm_bwd(dy) + dres, where dres is the gradient that reached h
// through the residual stream; the same dx is the gradient of both x and r.
std::vector<at::Tensor> add_rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w, const at::Tensor& rstd,
                                        const at::Tensor& dres) {
  CHECK_BF16(dres);
  TORCH_CHECK(dres.numel() == h.numel(), "add_rmsnorm_bwd: dres shape mismatch");
  return rmsnorm_bwd_impl(dy, h, w, rstd, bp(dres));
}

at::Tensor add_rmsnorm_bwd_into(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w, const at::Tensor& rstd,
                                const at::Tensor& dres, const at::Tensor& dw_out) {
  CHECK_BF16(dres);
  TORCH_CHECK(dres.numel() == h.numel(), "add_rmsnorm_bwd_into: dres shape mismatch");
  return rmsnorm_bwd_impl(dy, h, w, rstd, bp(dres), &dw_out)[0];
}

std::vector<at::Tensor> rmsnorm_bwd_impl(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd,
                                         const u16* dres, const at::Tensor* dw_out) {
  CHECK_BF16(dy);
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_F32(rstd);
  const int D = (int)x.size(-1);
  const int M = (int)(x.numel() / D);
  TORCH_CHECK(dy.numel() == x.numel() && rstd.numel() == M, "rmsnorm_bwd: shape mismatch");
  auto dx = at::empty_like(x);
  at::Tensor dw;
  if (dw_out) {
    CHECK_BF16(*dw_out);
    TORCH_CHECK(dw_out->numel() == D, "rmsnorm_bwd: dw_out must hold D elements");
    dw = *dw_out;
  } else {
    dw = at::empty({D}, w.options());
  }
  // 1024 waves (4 per CU) fill the chip; each takes M/1024 rows so the dW partials stay at 16 MB.
  // 2048 waves measured slower for the fused (ACC) variant at [16384, 4096]: 160.4 vs 143.5 us
  // (bench/norm_bench.py; the plain variant went 197 -> 171 us incl. its separate add).
  int grid = std::max(1, std::min((M + 3) / 4, 256));
  auto part = at::empty({(int64_t)grid * 4, D}, x.options().dtype(at::kFloat));
  if (M > 0) {
    const int nv = (D + 511) / 512;
    if (nv <= 1) rmsnorm_bwd_launch<1>(dy, x, w, rstd, dx, part, grid, M, D, dres);
    else if (nv <= 2) rmsnorm_bwd_launch<2>(dy, x, w, rstd, dx, part, grid, M, D, dres);
    else if (nv <= 4) rmsnorm_bwd_launch<4>(dy, x, w, rstd, dx, part, grid, M, D, dres);
    else if (nv <= 8) rmsnorm_bwd_launch<8>(dy, x, w, rstd, dx, part, grid, M, D, dres);
    else rmsnorm_bwd_launch<16>(dy, x, w, rstd, dx, part, grid, M, D, dres);
  } else {
    part.zero_();
  }
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((D + kColW - 1) / kColW), dim3(64 * kColWaves), 0, cur_stream(), part.data_ptr<float>(),
                     bpm(dw), grid * 4, D);
  return {dx, dw};
}

// =============================================================================== RoPE + QKV split
// qkv: [B*S, (H + 2*Hkv) * Dh] (token-major, the fused QKV GEMM output).  Outputs q [B,H,S,Dh],
// k [B,Hkv,S,Dh], v [B,Hkv,S,Dh].  Rotation (HF/Llama "rotate_half"): for i < Dh/2
//   out[i] = x[i]*cos - x[i+Dh/2]*sin ; out[i+Dh/2] = x[i+Dh/2]*cos + x[i]*sin
// cos/sin tables: fp32 [S_max, Dh/2].  One thread = 8 consecutive pairs of one (token, head).
// Backward (inverse=true) maps dq/dk/dv back to dqkv with the transposed rotation (sin -> -sin).
template <bool kInverse>
__global__ __launch_bounds__(256) void rope_split_kernel(u16* __restrict__ qkv, u16* __restrict__ q, u16* __restrict__ k,
                                                         u16* __restrict__ v, const float* __restrict__ cosb,
                                                         const float* __restrict__ sinb, int B, int S, int H, int Hkv,
                                                         int Dh, int pos_offset) {
  const int half = Dh >> 1;
  const int vec_per_head = half >> 3;  // threads per head (each covers 8 pairs)
  const int heads = H + 2 * Hkv;
  const size_t total = (size_t)B * S * heads * vec_per_head;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int vi = (int)(idx % vec_per_head);
    size_t t = idx / vec_per_head;
    const int hh = (int)(t % heads);
    t /= heads;  // token index
    const int s = (int)(t % S);
    const int b = (int)(t / S);
    u16* src = qkv + t * (size_t)heads * Dh + (size_t)hh * Dh;
    u16* dst;
    if (hh < H)
      dst = q + (((size_t)b * H + hh) * S + s) * Dh;
    else if (hh < H + Hkv)
      dst = k + (((size_t)b * Hkv + (hh - H)) * S + s) * Dh;
    else
      dst = v + (((size_t)b * Hkv + (hh - H - Hkv)) * S + s) * Dh;
    const int i0 = vi * 8;
    u16* fa = kInverse ? dst : src;  // read side
    u16* ta = kInverse ? src : dst;  // write side
    u16x8 lo = *reinterpret_cast<const u16x8*>(fa + i0);
    u16x8 hi = *reinterpret_cast<const u16x8*>(fa + half + i0);
    if (hh >= H + Hkv) {  // V: plain copy
      *reinterpret_cast<u16x8*>(ta + i0) = lo;
      *reinterpret_cast<u16x8*>(ta + half + i0) = hi;
      continue;
    }
    const float* cr = cosb + (size_t)(s + pos_offset) * half + i0;
    const float* sr = sinb + (size_t)(s + pos_offset) * half + i0;
    f32x4 c0 = *reinterpret_cast<const f32x4*>(cr), c1 = *reinterpret_cast<const f32x4*>(cr + 4);
    f32x4 s0 = *reinterpret_cast<const f32x4*>(sr), s1 = *reinterpret_cast<const f32x4*>(sr + 4);
    u16x8 olo, ohi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4];
      const float sn = (j < 4 ? s0[j] : s1[j - 4]) * (kInverse ? -1.f : 1.f);
      const float a = bf2f(lo[j]), bb = bf2f(hi[j]);
      olo[j] = f2bf(a * c - bb * sn);
      ohi[j] = f2bf(bb * c + a * sn);
    }
    *reinterpret_cast<u16x8*>(ta + i0) = olo;
    *reinterpret_cast<u16x8*>(ta + half + i0) = ohi;
  }
}

int grid_for(size_t work, int per_block = 256) {
  size_t g = (work + per_block - 1) / per_block;
  return (int)std::max<size_t>(1, std::min<size_t>(g, 256 * 16));  // >> 256 CUs, grid-stride beyond
}

std::vector<at::Tensor> rope_split_fwd(const at::Tensor& qkv, const at::Tensor& cosb, const at::Tensor& sinb, int64_t B,
                                       int64_t S, int64_t H, int64_t Hkv, int64_t Dh, int64_t pos_offset) {
  CHECK_BF16(qkv);
  CHECK_F32(cosb);
  CHECK_F32(sinb);
  TORCH_CHECK(Dh % 16 == 0, "head dim must be a multiple of 16");
  TORCH_CHECK(qkv.numel() == B * S * (H + 2 * Hkv) * Dh, "qkv shape mismatch");
  TORCH_CHECK(cosb.size(-1) == Dh / 2 && cosb.size(0) >= S + pos_offset && sinb.sizes() == cosb.sizes(), "rope table shape");
  auto opt = qkv.options();
  auto q = at::empty({B, H, S, Dh}, opt), k = at::empty({B, Hkv, S, Dh}, opt), v = at::empty({B, Hkv, S, Dh}, opt);
  const size_t work = (size_t)B * S * (H + 2 * Hkv) * (Dh / 16);
  if (work)
    hipLaunchKernelGGL(rope_split_kernel<false>, dim3(grid_for(work)), dim3(256), 0, cur_stream(),
                       const_cast<u16*>(bp(qkv)), bpm(q), bpm(k), bpm(v), cosb.data_ptr<float>(), sinb.data_ptr<float>(),
                       (int)B, (int)S, (int)H, (int)Hkv, (int)Dh, (int)pos_offset);
  return {q, k, v};
}

at::Tensor rope_split_bwd(const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, const at::Tensor& cosb,
                          const at::Tensor& sinb, int64_t pos_offset) {
  CHECK_BF16(dq);
  CHECK_BF16(dk);
  CHECK_BF16(dv);
  const int64_t B = dq.size(0), H = dq.size(1), S = dq.size(2), Dh = dq.size(3), Hkv = dk.size(1);
  auto dqkv = at::empty({B * S, (H + 2 * Hkv) * Dh}, dq.options());
  const size_t work = (size_t)B * S * (H + 2 * Hkv) * (Dh / 16);
  if (work)
    hipLaunchKernelGGL(rope_split_kernel<true>, dim3(grid_for(work)), dim3(256), 0, cur_stream(), bpm(dqkv),
                       const_cast<u16*>(bp(dq)), const_cast<u16*>(bp(dk)), const_cast<u16*>(bp(dv)), cosb.data_ptr<float>(),
                       sinb.data_ptr<float>(), (int)B, (int)S, (int)H, (int)Hkv, (int)Dh, (int)pos_offset);
  return dqkv;
}

// RoPE backward with a transposed copy: dqkv^T [(H+2Hkv)*128, B*S] is the A operand of the QKV
// weight-gradient GEMM in NT layout, written from the LDS tile instead of by a transpose pass that
// re-reads dqkv.  One 256-thread block = 64 tokens x one head (head dim 128): a thread takes 8
// rotation pairs (lo = x[8v..8v+7], hi = x[64+8v..]) of one token, the tile is staged in LDS with the
// swiglu_bwd_t128 swizzle and written as 128-B segments of the transposed rows.  Same expressions as
// rope_split_kernel<true> (bit-identical dqkv).  S multiple of 64.
__global__ __launch_bounds__(256) void rope_bwd_t_kernel(u16* __restrict__ dqkv, u16* __restrict__ dqkvT,
                                                         const u16* __restrict__ q, const u16* __restrict__ k,
                                                         const u16* __restrict__ v, const float* __restrict__ cosb,
                                                         const float* __restrict__ sinb, int B, int S, int H, int Hkv,
                                                         int pos_offset) {
  constexpr int Dh = 128, half = 64;
  __shared__ u16x8 tile[64][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int hh = blockIdx.x, heads = H + 2 * Hkv;
  const size_t tok0 = (size_t)blockIdx.y * 64;  // never crosses a sequence (S % 64 == 0)
  const int b = (int)(tok0 / S), s0 = (int)(tok0 % S);
  const u16* src;
  if (hh < H) src = q + (((size_t)b * H + hh) * S + s0) * Dh;
  else if (hh < H + Hkv) src = k + (((size_t)b * Hkv + (hh - H)) * S + s0) * Dh;
  else src = v + (((size_t)b * Hkv + (hh - H - Hkv)) * S + s0) * Dh;
  const int vi = t & 7;
  u16x8 lol[2], hil[2];  // both passes' loads first (as swiglu_bwd_t128_kernel)
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const u16* fa = src + (size_t)((t >> 3) + 32 * pass) * Dh;
    lol[pass] = *reinterpret_cast<const u16x8*>(fa + vi * 8);
    hil[pass] = *reinterpret_cast<const u16x8*>(fa + half + vi * 8);
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int r = (t >> 3) + 32 * pass;
    const int i0 = vi * 8;
    const u16x8 lo = lol[pass];
    const u16x8 hi = hil[pass];
    u16x8 olo, ohi;
    if (hh >= H + Hkv) {  // V: plain copy
      olo = lo;
      ohi = hi;
    } else {
      const int sp = s0 + r;
      const float* cr = cosb + (size_t)(sp + pos_offset) * half + i0;
      const float* sr = sinb + (size_t)(sp + pos_offset) * half + i0;
      f32x4 c0 = *reinterpret_cast<const f32x4*>(cr), c1 = *reinterpret_cast<const f32x4*>(cr + 4);
      f32x4 sn0 = *reinterpret_cast<const f32x4*>(sr), sn1 = *reinterpret_cast<const f32x4*>(sr + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = j < 4 ? c0[j] : c1[j - 4];
        const float sn = (j < 4 ? sn0[j] : sn1[j - 4]) * -1.f;
        const float a = bf2f(lo[j]), bb = bf2f(hi[j]);
        olo[j] = f2bf(a * c - bb * sn);
        ohi[j] = f2bf(bb * c + a * sn);
      }
    }
    u16* ta = dqkv + (tok0 + r) * (size_t)heads * Dh + (size_t)hh * Dh;
    *reinterpret_cast<u16x8*>(ta + i0) = olo;
    *reinterpret_cast<u16x8*>(ta + half + i0) = ohi;
    tile[r][vi ^ ((r >> 3) & 7)] = olo;
    tile[r][(8 + vi) ^ ((r >> 3) & 7)] = ohi;
  }
  __syncthreads();
  const size_t BS = (size_t)B * S;
  const int p = lane >> 3, cl = lane & 7;
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int vc = 4 * i + wv;
    const int c = 8 * vc + cl;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[((8 * p + j) * 16 + (vc ^ p)) * 8 + cl];
    *reinterpret_cast<u16x8*>(dqkvT + ((size_t)hh * Dh + c) * BS + tok0 + 8 * p) = o;
  }
}

// rope_split_bwd that also returns dqkv^T [(H+2Hkv)*Dh, B*S]; head dim 128, S multiple of 64
std::vector<at::Tensor> rope_split_bwd_t(const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, const at::Tensor& cosb,
                                         const at::Tensor& sinb, int64_t pos_offset) {
  CHECK_BF16(dq);
  CHECK_BF16(dk);
  CHECK_BF16(dv);
  CHECK_F32(cosb);
  CHECK_F32(sinb);
  const int64_t B = dq.size(0), H = dq.size(1), S = dq.size(2), Dh = dq.size(3), Hkv = dk.size(1);
  TORCH_CHECK(Dh == 128 && S % 64 == 0, "rope_split_bwd_t: head dim 128 and S multiple of 64");
  TORCH_CHECK(dk.sizes() == dv.sizes() && dk.size(0) == B && dk.size(2) == S && dk.size(3) == Dh, "rope_split_bwd_t: shapes");
  TORCH_CHECK(cosb.size(-1) == Dh / 2 && cosb.size(0) >= S + pos_offset && sinb.sizes() == cosb.sizes(), "rope table shape");
  TORCH_CHECK(B * S / 64 <= 65535, "rope_split_bwd_t: too many tokens for the grid");
  const int64_t heads = H + 2 * Hkv;
  auto dqkv = at::empty({B * S, heads * Dh}, dq.options());
  auto dqkvT = at::empty({heads * Dh, B * S}, dq.options());
  if (B * S)
    hipLaunchKernelGGL(rope_bwd_t_kernel, dim3((unsigned)heads, (unsigned)(B * S / 64)), dim3(256), 0, cur_stream(), bpm(dqkv),
                       bpm(dqkvT), bp(dq), bp(dk), bp(dv), cosb.data_ptr<float>(), sinb.data_ptr<float>(), (int)B, (int)S, (int)H,
                       (int)Hkv, (int)pos_offset);
  return {dqkv, dqkvT};
}

// =============================================================================== SwiGLU
// gu: [T, 2F] = [gate | up]; h = silu(g) * u : [T, F]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const u16* __restrict__ gu, u16* __restrict__ h, size_t T, int F) {
  const int fv = F >> 3;
  const size_t total = T * fv;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t t = i / fv;
    const int c = (int)(i % fv);
    const u16x8 g = reinterpret_cast<const u16x8*>(gu + t * 2 * F)[c];
    const u16x8 u = reinterpret_cast<const u16x8*>(gu + t * 2 * F + F)[c];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      o[j] = f2bf(gf / (1.f + __expf(-gf)) * bf2f(u[j]));
    }
    reinterpret_cast<u16x8*>(h + t * F)[c] = o;
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const u16* __restrict__ dh, const u16* __restrict__ gu,
                                                         u16* __restrict__ dgu, size_t T, int F) {
  const int fv = F >> 3;
  const size_t total = T * fv;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t t = i / fv;
    const int c = (int)(i % fv);
    const u16x8 g = reinterpret_cast<const u16x8*>(gu + t * 2 * F)[c];
    const u16x8 u = reinterpret_cast<const u16x8*>(gu + t * 2 * F + F)[c];
    const u16x8 d = reinterpret_cast<const u16x8*>(dh + t * F)[c];
    u16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      const float sg = 1.f / (1.f + __expf(-gf));
      const float silu = gf * sg;
      ou[j] = f2bf(df * silu);
      og[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    reinterpret_cast<u16x8*>(dgu + t * 2 * F)[c] = og;
    reinterpret_cast<u16x8*>(dgu + t * 2 * F + F)[c] = ou;
  }
}

// Backward with a second, transposed copy of the gradient: dguT [2F, T] is the A operand of the
// w13 weight-gradient GEMM in NT layout (dW13 = dguT . hT^T), written here from the LDS tile instead
// of by a separate transpose pass (saves re-reading the 2*T*F gradient).  One 256-thread block =
// 64 tokens x 64 features: each thread computes 2 x 8 features of the gate AND up halves, stores
// them row-major, stages both tiles in LDS (XOR-swizzled exactly like csrc/ops/transpose.hip) and
// writes 2 x 8 tokens of a transposed row per tile.  T and F must be multiples of 64.
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const u16* __restrict__ dh, const u16* __restrict__ gu,
                                                           u16* __restrict__ dgu, u16* __restrict__ dguT, int T, int F) {
  __shared__ u16x8 tile[2][64][8];  // [gate | up][token][feature vector]
  const int t = threadIdx.x;
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 64;
  const size_t F2 = 2 * (size_t)F;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (t >> 3) + 32 * i, v = t & 7;
    const size_t row = r0 + r;
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + row * F2 + c0 + 8 * v);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + row * F2 + F + c0 + 8 * v);
    const u16x8 d = *reinterpret_cast<const u16x8*>(dh + row * F + c0 + 8 * v);
    u16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      const float sg = 1.f / (1.f + __expf(-gf));
      const float silu = gf * sg;  // same expression order as swiglu_bwd_kernel: identical rounding
      ou[j] = f2bf(df * silu);
      og[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    *reinterpret_cast<u16x8*>(dgu + row * F2 + c0 + 8 * v) = og;
    *reinterpret_cast<u16x8*>(dgu + row * F2 + F + c0 + 8 * v) = ou;
    tile[0][r][v ^ ((r >> 3) & 7)] = og;
    tile[1][r][v ^ ((r >> 3) & 7)] = ou;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u16* lds = reinterpret_cast<const u16*>(&tile[h][0][0]);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = t + 256 * i;
      const int c = idx >> 3, p = idx & 7;
      const int pv = (c >> 3) ^ p;
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = lds[(8 * p + j) * 64 + pv * 8 + (c & 7)];
      *reinterpret_cast<u16x8*>(dguT + ((size_t)h * F + c0 + c) * T + r0 + 8 * p) = o;
    }
  }
}

// Forward with a transposed copy of the output: hT [F, T] is the B operand of the w2 weight-gradient
// GEMM in NT layout, written from the LDS tile here (Llama(transpose_x="forward")) instead of by a
// transpose pass over the 2*T*F-byte output in the backward.  Same tiling and swizzle as
// swiglu_bwd_t_kernel, same expression as swiglu_fwd_kernel (identical h bits).  T, F multiples of 64.
__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const u16* __restrict__ gu, u16* __restrict__ h,
                                                           u16* __restrict__ hT, int T, int F) {
  __shared__ u16x8 tile[64][8];
  const int t = threadIdx.x;
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 64;
  const size_t F2 = 2 * (size_t)F;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (t >> 3) + 32 * i, v = t & 7;
    const size_t row = r0 + r;
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + row * F2 + c0 + 8 * v);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + row * F2 + F + c0 + 8 * v);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      o[j] = f2bf(gf / (1.f + __expf(-gf)) * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(h + row * F + c0 + 8 * v) = o;
    tile[r][v ^ ((r >> 3) & 7)] = o;
  }
  __syncthreads();
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i;
    const int c = idx >> 3, p = idx & 7;
    const int pv = (c >> 3) ^ p;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[(8 * p + j) * 64 + pv * 8 + (c & 7)];
    *reinterpret_cast<u16x8*>(hT + (c0 + c) * T + r0 + 8 * p) = o;
  }
}

std::vector<at::Tensor> swiglu_fwd_t(const at::Tensor& gu) {
  CHECK_BF16(gu);
  TORCH_CHECK(gu.dim() == 2, "swiglu_fwd_t: gu must be [T, 2F]");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(T % 64 == 0 && F % 64 == 0 && T / 64 <= 65535, "swiglu_fwd_t: T and F must be multiples of 64");
  auto h = at::empty({T, F}, gu.options());
  auto hT = at::empty({F, T}, gu.options());
  if (T && F) hipLaunchKernelGGL(swiglu_fwd_t_kernel, dim3((unsigned)(F / 64), (unsigned)(T / 64)), dim3(256), 0, cur_stream(), bp(gu),
                           bpm(h), bpm(hT), (int)T, (int)F);
  return {h, hT};
}

// swiglu_fwd_t with 64-token x 128-feature tiles (the swiglu_bwd_t128 layout): 256-B row segments of
// gate / up / h, 128-B segments of the transposed rows, conflict-free transposed LDS reads.  Same
// expression as swiglu_fwd_kernel (identical h bits).  T multiple of 64, F multiple of 128.
__global__ __launch_bounds__(256) void swiglu_fwd_t128_kernel(const u16* __restrict__ gu, u16* __restrict__ h,
                                                              u16* __restrict__ hT, int T, int F) {
  __shared__ u16x8 tile[64][16];  // [token][feature vector, swizzled]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 128;
  const size_t F2 = 2 * (size_t)F;
  u16x8 gl[4], ul[4];  // all 8 loads of the tile first (as swiglu_bwd_t128_kernel)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const size_t row = r0 + (t >> 4) + 16 * i;
    const int v = t & 15;
    gl[i] = *reinterpret_cast<const u16x8*>(gu + row * F2 + c0 + 8 * v);
    ul[i] = *reinterpret_cast<const u16x8*>(gu + row * F2 + F + c0 + 8 * v);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i, v = t & 15;
    const size_t row = r0 + r;
    const u16x8 g = gl[i], u = ul[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      o[j] = f2bf(gf / (1.f + __expf(-gf)) * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(h + row * F + c0 + 8 * v) = o;
    tile[r][v ^ ((r >> 3) & 7)] = o;
  }
  __syncthreads();
  const int p = lane >> 3, cl = lane & 7;
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int vc = 4 * i + wv;
    const int c = 8 * vc + cl;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[((8 * p + j) * 16 + (vc ^ p)) * 8 + cl];
    *reinterpret_cast<u16x8*>(hT + (c0 + c) * T + r0 + 8 * p) = o;
  }
}

std::vector<at::Tensor> swiglu_fwd_t128(const at::Tensor& gu) {
  CHECK_BF16(gu);
  TORCH_CHECK(gu.dim() == 2, "swiglu_fwd_t128: gu must be [T, 2F]");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(T % 64 == 0 && F % 128 == 0 && T / 64 <= 65535, "swiglu_fwd_t128: T multiple of 64, F of 128");
  auto h = at::empty({T, F}, gu.options());
  auto hT = at::empty({F, T}, gu.options());
  if (T && F) hipLaunchKernelGGL(swiglu_fwd_t128_kernel, dim3((unsigned)(F / 128), (unsigned)(T / 64)), dim3(256), 0, cur_stream(),
                           bp(gu), bpm(h), bpm(hT), (int)T, (int)F);
  return {h, hT};
}

// swiglu_bwd_t with 64-token x 128-feature tiles: 256-B row segments of dh / gate / up (the 64 x 64
// tile reads 128-B segments and ran at 4.96 TB/s in the Llama step, profiles/r04_llama) and 128-B
// segments of the transposed rows.  Lanes of one transposed-store instruction take one 16-B column
// vector x 8 row groups (the swizzle puts the row groups on 8 slots): conflict-free.  Same arithmetic
// as swiglu_bwd_kernel (bit-identical).  T multiple of 64, F multiple of 128.
__global__ __launch_bounds__(256) void swiglu_bwd_t128_kernel(const u16* __restrict__ dh, const u16* __restrict__ gu,
                                                              u16* __restrict__ dgu, u16* __restrict__ dguT, int T, int F) {
  __shared__ u16x8 tile[2][64][16];  // [gate | up][token][feature vector, swizzled]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 128;
  const size_t F2 = 2 * (size_t)F;
  // all 12 loads of the tile first (the compiler otherwise issued one pass's 3 loads and waited for
  // them before the next pass: 48 B per lane in flight, 5.2 TB/s)
  u16x8 gl[4], ul[4], dl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const size_t row = r0 + (t >> 4) + 16 * i;
    const int v = t & 15;
    gl[i] = *reinterpret_cast<const u16x8*>(gu + row * F2 + c0 + 8 * v);
    ul[i] = *reinterpret_cast<const u16x8*>(gu + row * F2 + F + c0 + 8 * v);
    dl[i] = *reinterpret_cast<const u16x8*>(dh + row * F + c0 + 8 * v);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i, v = t & 15;
    const size_t row = r0 + r;
    const u16x8 g = gl[i], u = ul[i], d = dl[i];
    u16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      const float sg = 1.f / (1.f + __expf(-gf));
      const float silu = gf * sg;
      ou[j] = f2bf(df * silu);
      og[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    *reinterpret_cast<u16x8*>(dgu + row * F2 + c0 + 8 * v) = og;
    *reinterpret_cast<u16x8*>(dgu + row * F2 + F + c0 + 8 * v) = ou;
    tile[0][r][v ^ ((r >> 3) & 7)] = og;
    tile[1][r][v ^ ((r >> 3) & 7)] = ou;
  }
  __syncthreads();
  const int p = lane >> 3, cl = lane & 7;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u16* lds = reinterpret_cast<const u16*>(&tile[h][0][0]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int vc = 4 * i + wv;
      const int c = 8 * vc + cl;
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = lds[((8 * p + j) * 16 + (vc ^ p)) * 8 + cl];
      *reinterpret_cast<u16x8*>(dguT + ((size_t)h * F + c0 + c) * T + r0 + 8 * p) = o;
    }
  }
}

std::vector<at::Tensor> swiglu_bwd_t128(const at::Tensor& dh, const at::Tensor& gu) {
  CHECK_BF16(dh);
  CHECK_BF16(gu);
  TORCH_CHECK(gu.dim() == 2, "swiglu_bwd_t128: gu must be [T, 2F]");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(dh.numel() == T * F, "swiglu_bwd_t128: shape mismatch");
  TORCH_CHECK(T % 64 == 0 && F % 128 == 0 && T / 64 <= 65535, "swiglu_bwd_t128: T multiple of 64, F of 128");
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({2 * F, T}, gu.options());
  if (T && F) hipLaunchKernelGGL(swiglu_bwd_t128_kernel, dim3((unsigned)(F / 128), (unsigned)(T / 64)), dim3(256), 0, cur_stream(),
                           bp(dh), bp(gu), bpm(dgu), bpm(dguT), (int)T, (int)F);
  return {dgu, dguT};
}

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  CHECK_BF16(gu);
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: 2F must be a multiple of 16");
  const int F = (int)(F2 / 2);
  const size_t T = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto h = at::empty(sizes, gu.options());
  if (T) hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(T * (F / 8))), dim3(256), 0, cur_stream(), bp(gu), bpm(h), T, F);
  return h;
}

at::Tensor swiglu_bwd(const at::Tensor& dh, const at::Tensor& gu) {
  CHECK_BF16(dh);
  CHECK_BF16(gu);
  const int F = (int)(gu.size(-1) / 2);
  const size_t T = gu.numel() / (2 * F);
  TORCH_CHECK((size_t)dh.numel() == T * F, "swiglu_bwd: shape mismatch");
  auto dgu = at::empty_like(gu);
  if (T) hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(T * (F / 8))), dim3(256), 0, cur_stream(), bp(dh), bp(gu), bpm(dgu), T, F);
  return dgu;
}

std::vector<at::Tensor> swiglu_bwd_t(const at::Tensor& dh, const at::Tensor& gu) {
  CHECK_BF16(dh);
  CHECK_BF16(gu);
  TORCH_CHECK(gu.dim() == 2, "swiglu_bwd_t: gu must be [T, 2F]");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(dh.numel() == T * F, "swiglu_bwd_t: shape mismatch");
  TORCH_CHECK(T % 64 == 0 && F % 64 == 0 && T / 64 <= 65535, "swiglu_bwd_t: T and F must be multiples of 64");
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({2 * F, T}, gu.options());
  if (T && F) hipLaunchKernelGGL(swiglu_bwd_t_kernel, dim3((unsigned)(F / 64), (unsigned)(T / 64)), dim3(256), 0, cur_stream(), bp(dh),
                           bp(gu), bpm(dgu), bpm(dguT), (int)T, (int)F);
  return {dgu, dguT};
}

// =============================================================================== cross-entropy
// One 256-thread block per row; online (max, sum-exp) over 16-B vectors, block reduce through LDS.
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mx = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mx)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mx));
  m = mx;
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse, int V,
                                                       int64_t ignore_index) {
  __shared__ float sm[4], ss[4];
  const int row = blockIdx.x;
  const u16x8* lr = reinterpret_cast<const u16x8*>(logits + (size_t)row * V);
  const int nvec = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nvec; c += 256) {
    const u16x8 x = lr[c];
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) lm = fmaxf(lm, bf2f(x[j]));
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(bf2f(x[j]) - lm);
    online_merge(m, s, lm, ls);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
    online_merge(m, s, m2, s2);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[wave] = m;
    ss[wave] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int w = 1; w < 4; ++w) online_merge(M, Ssum, sm[w], ss[w]);
    const float l = M + __logf(Ssum);
    lse[row] = l;
    const int64_t y = labels[row];
    loss[row] = (y == ignore_index || y < 0 || y >= V) ? 0.f : l - bf2f(logits[(size_t)row * V + y]);
  }
}

// dlogits = (softmax - onehot) * scale, written over the logits (scale = dL/dloss_mean per valid row)
__global__ __launch_bounds__(256) void xent_bwd_kernel(u16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ gscale,
                                                       int V, int64_t ignore_index) {
  const int row = blockIdx.x;
  const int64_t y = labels[row];
  const bool ignored = (y == ignore_index || y < 0 || y >= V);
  const float l = lse[row];
  const float sc = ignored ? 0.f : gscale[0];
  u16x8* lr = reinterpret_cast<u16x8*>(logits + (size_t)row * V);
  const int nvec = V >> 3;
  for (int c = threadIdx.x; c < nvec; c += 256) {
    const u16x8 x = lr[c];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      const float p = __expf(bf2f(x[j]) - l);
      o[j] = f2bf((p - (col == y ? 1.f : 0.f)) * sc);
    }
    lr[c] = o;
  }
}

// xent_bwd with a transposed copy: dlogits^T [V, T] is the A operand of the lm_head weight-gradient
// GEMM in NT layout, written from the LDS tile instead of by a transpose pass that re-reads the
// 4.2 GB gradient (Llama-3-8B, T 16384).  One 256-thread block = 64 rows x 128 vocabulary columns:
// 256-B row segments in, 128-B transposed segments out (the swiglu_bwd_t128 tile).  Same expression
// as xent_bwd_kernel (bit-identical dlogits).  T multiple of 64, V multiple of 128.
__global__ __launch_bounds__(256) void xent_bwd_t_kernel(u16* __restrict__ logits, u16* __restrict__ dlT,
                                                         const int64_t* __restrict__ labels, const float* __restrict__ lse,
                                                         const float* __restrict__ gscale, int T, int V, int64_t ignore_index) {
  __shared__ u16x8 tile[64][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const size_t r0 = (size_t)blockIdx.y * 64, c0 = (size_t)blockIdx.x * 128;
  const float g = gscale[0];
  u16x8 xl[4];  // the tile's 4 loads first (as swiglu_bwd_t128_kernel)
#pragma unroll
  for (int i = 0; i < 4; ++i) xl[i] = *reinterpret_cast<const u16x8*>(logits + (r0 + (t >> 4) + 16 * i) * V + c0 + 8 * (t & 15));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (t >> 4) + 16 * i, v = t & 15;
    const size_t row = r0 + r;
    const int64_t y = labels[row];
    const bool ignored = (y == ignore_index || y < 0 || y >= V);
    const float l = lse[row];
    const float sc = ignored ? 0.f : g;
    u16x8* src = reinterpret_cast<u16x8*>(logits + row * V + c0 + 8 * v);
    const u16x8 x = xl[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t col = (int64_t)c0 + 8 * v + j;
      const float p = __expf(bf2f(x[j]) - l);
      o[j] = f2bf((p - (col == y ? 1.f : 0.f)) * sc);
    }
    *src = o;
    tile[r][v ^ ((r >> 3) & 7)] = o;
  }
  __syncthreads();
  const int p = lane >> 3, cl = lane & 7;
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int vc = 4 * i + wv;
    const int c = 8 * vc + cl;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[((8 * p + j) * 16 + (vc ^ p)) * 8 + cl];
    *reinterpret_cast<u16x8*>(dlT + (c0 + c) * T + r0 + 8 * p) = o;
  }
}

std::vector<at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& labels, int64_t ignore_index) {
  CHECK_BF16(logits);
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous(), "labels must be int64 GPU");
  const int V = (int)logits.size(-1);
  TORCH_CHECK(V % 8 == 0, "vocab must be a multiple of 8");
  const int64_t T = logits.numel() / V;
  TORCH_CHECK(labels.numel() == T, "labels/logits mismatch");
  auto loss = at::empty({T}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({T}, logits.options().dtype(at::kFloat));
  if (T) hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)T), dim3(256), 0, cur_stream(), bp(logits), labels.data_ptr<int64_t>(),
                            loss.data_ptr<float>(), lse.data_ptr<float>(), V, ignore_index);
  return {loss, lse};
}

void xent_bwd_inplace(at::Tensor& logits, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& gscale,
                      int64_t ignore_index) {
  CHECK_BF16(logits);
  CHECK_F32(lse);
  CHECK_F32(gscale);
  const int V = (int)logits.size(-1);
  const int64_t T = logits.numel() / V;
  if (T) hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)T), dim3(256), 0, cur_stream(), bpm(logits), labels.data_ptr<int64_t>(),
                            lse.data_ptr<float>(), gscale.data_ptr<float>(), V, ignore_index);
}

// dlogits in place over the logits AND its transpose [V, T] (returned).  T multiple of 64, V of 128.
at::Tensor xent_bwd_t(at::Tensor& logits, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& gscale,
                      int64_t ignore_index) {
  CHECK_BF16(logits);
  CHECK_F32(lse);
  CHECK_F32(gscale);
  TORCH_CHECK(logits.dim() == 2, "xent_bwd_t: logits must be [T, V]");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous(), "labels must be int64 GPU");
  const int64_t T = logits.size(0), V = logits.size(1);
  TORCH_CHECK(labels.numel() == T && lse.numel() == T, "xent_bwd_t: labels/lse must have T entries");
  TORCH_CHECK(T % 64 == 0 && V % 128 == 0 && T / 64 <= 65535, "xent_bwd_t: T multiple of 64, V of 128");
  auto dlT = at::empty({V, T}, logits.options());
  if (T && V)
    hipLaunchKernelGGL(xent_bwd_t_kernel, dim3((unsigned)(V / 128), (unsigned)(T / 64)), dim3(256), 0, cur_stream(), bpm(logits),
                       bpm(dlT), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), gscale.data_ptr<float>(), (int)T, (int)V,
                       ignore_index);
  return dlT;
}

// =============================================================================== embedding backward
// dW_emb[tok] = sum of the dx rows of every position holding tok, written straight into the weight's
// slot of the flat gradient buffer (rows no position holds are zeroed by the caller).  The positions
// arrive sorted by token (stable: equal tokens in position order), so one wave per segment start sums
// its segment in a fixed order in fp32 and rounds once: deterministic, no atomics.  Replaces torch's
// embedding backward (sort + two kernels + a dense [V, D] gradient) and autograd's add of that
// dense gradient into the flat buffer.
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                                                        const u16* __restrict__ dx, u16* __restrict__ out, int T, int D,
                                                        int64_t V) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= T) return;
  const int64_t tok = sorted[i];
  if ((i > 0 && sorted[i - 1] == tok) || tok < 0 || tok >= V) return;
  int end = i + 1;
  while (end < T && sorted[end] == tok) ++end;
  const int nvec = D >> 3;
  for (int c = lane; c < nvec; c += 64) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = i; j < end; ++j) {
      const u16x8 x = reinterpret_cast<const u16x8*>(dx + (size_t)perm[j] * D)[c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(x[e]);
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    reinterpret_cast<u16x8*>(out + (size_t)tok * D)[c] = o;
  }
}

// out: [V, D] bf16 (contiguous view), zeroed by the caller; sorted / perm: int64 [T]; dx: bf16 [T, D]
void embed_bwd_into(const at::Tensor& sorted, const at::Tensor& perm, const at::Tensor& dx, at::Tensor& out) {
  CHECK_BF16(dx);
  CHECK_BF16(out);
  TORCH_CHECK(sorted.is_cuda() && perm.is_cuda() && sorted.scalar_type() == at::kLong && perm.scalar_type() == at::kLong &&
                  sorted.is_contiguous() && perm.is_contiguous(), "embed_bwd_into: sorted / perm must be contiguous int64 GPU tensors");
  TORCH_CHECK(dx.dim() == 2 && out.dim() == 2 && dx.size(1) == out.size(1) && dx.size(1) % 8 == 0, "embed_bwd_into: shapes");
  const int64_t T = dx.size(0);
  TORCH_CHECK(sorted.numel() == T && perm.numel() == T && T < (int64_t(1) << 31), "embed_bwd_into: sorted / perm must have T entries");
  if (T)
    hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, cur_stream(), sorted.data_ptr<int64_t>(),
                       perm.data_ptr<int64_t>(), bp(dx), bpm(out), (int)T, (int)dx.size(1), out.size(0));
}

// =============================================================================== optimizer
// Flat-buffer AdamW (decoupled weight decay).  8 elements per thread per iteration: two 16-B loads
// each of master/m/v, one 16-B load of the bf16 gradient; writes master/m/v and the bf16 weight.
// hp: device fp32 [lr, beta1, beta2, eps, weight_decay, grad_scale, bias_c1, bias_c2] so a captured
// graph replays with updated hyper-parameters.
// 8 gradient elements of vector i as fp32: the bf16 gradient buffer, or the fp32 buffer a DP
// all-reduce in fp32 leaves (parallel/dp.py grad_reduce="fp32")
__device__ __forceinline__ void load_g8(const u16* __restrict__ g, size_t i, float (&out)[8]) {
  const u16x8 gv = reinterpret_cast<const u16x8*>(g)[i];
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bf2f(gv[j]);
}
__device__ __forceinline__ void load_g8(const float* __restrict__ g, size_t i, float (&out)[8]) {
  const f32x4 a = reinterpret_cast<const f32x4*>(g)[2 * i], b = reinterpret_cast<const f32x4*>(g)[2 * i + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = a[j], out[j + 4] = b[j];
}

template <typename G>
__device__ __forceinline__ void adamw_body(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                           const G* __restrict__ g, u16* __restrict__ w, size_t n, float lr, float b1,
                                           float b2, float eps, float wd, float gs, float bc1, float bc2) {
  const size_t nv = n >> 3;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
    f32x4 p0 = reinterpret_cast<f32x4*>(master)[2 * i], p1 = reinterpret_cast<f32x4*>(master)[2 * i + 1];
    f32x4 m0 = reinterpret_cast<f32x4*>(m)[2 * i], m1 = reinterpret_cast<f32x4*>(m)[2 * i + 1];
    f32x4 v0 = reinterpret_cast<f32x4*>(v)[2 * i], v1 = reinterpret_cast<f32x4*>(v)[2 * i + 1];
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
      const float gr = gf[j] * gs;
      mm[j] = b1 * mm[j] + (1.f - b1) * gr;
      vv[j] = b2 * vv[j] + (1.f - b2) * gr * gr;
      const float upd = (mm[j] / bc1) / (sqrtf(vv[j] / bc2) + eps);
      p[j] = p[j] - lr * (upd + wd * p[j]);
      wo[j] = f2bf(p[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[j] = p[j], p1[j] = p[j + 4];
      m0[j] = mm[j], m1[j] = mm[j + 4];
      v0[j] = vv[j], v1[j] = vv[j + 4];
    }
    reinterpret_cast<f32x4*>(master)[2 * i] = p0;
    reinterpret_cast<f32x4*>(master)[2 * i + 1] = p1;
    reinterpret_cast<f32x4*>(m)[2 * i] = m0;
    reinterpret_cast<f32x4*>(m)[2 * i + 1] = m1;
    reinterpret_cast<f32x4*>(v)[2 * i] = v0;
    reinterpret_cast<f32x4*>(v)[2 * i + 1] = v1;
    reinterpret_cast<u16x8*>(w)[i] = wo;
  }
}

template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                                    const G* __restrict__ g, u16* __restrict__ w, const float* __restrict__ hp,
                                                    size_t n) {
  adamw_body(master, m, v, g, w, n, hp[0], hp[1], hp[2], hp[3], hp[4], hp[5], hp[6], hp[7]);
}

// Graph-mode AdamW: everything the host used to compute per step is derived on the device, so one
// captured launch replays correctly forever (``FlatAdamW(capturable=True)``).
//   hp   = [lr, beta1, beta2, eps, weight_decay, grad_scale, clip_norm (<= 0: off), -]
//   part = sqnorm partials of the gradient (``sq_norm_parts``); every block reduces them itself
//   t    = optimizer step count AFTER this step (``sq_norm_parts`` advanced it in stream order)
// Bias corrections 1 - beta^t and the clipping factor min(1, clip / ||g * grad_scale||) follow.
template <typename G>
__global__ __launch_bounds__(256) void adamw_dev_kernel(float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                                                        const G* __restrict__ g, u16* __restrict__ w, const float* __restrict__ hp,
                                                        const float* __restrict__ part, int nparts, const float* __restrict__ tptr,
                                                        size_t n) {
  __shared__ float red[4];
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], gscale = hp[5], clip = hp[6];
  float gs = gscale;
  if (nparts > 0 && clip > 0.f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * gscale;
    gs = gscale * fminf(1.f, clip / (norm + 1e-6f));
  }
  const float t = tptr[0];
  adamw_body(master, m, v, g, w, n, lr, b1, b2, eps, wd, gs, 1.f - powf(b1, t), 1.f - powf(b2, t));
}

// sum of squares of a bf16 buffer -> per-block partials (fp32)
template <typename G>
__global__ __launch_bounds__(256) void sqnorm_kernel(const G* __restrict__ g, float* __restrict__ part, size_t n) {
  __shared__ float red[4];
  // each thread's grid-stride vectors are loaded four at a time (four 16-B loads in flight per lane;
  // one at a time ran the 16 GB bf16 gradient at 5.3 TB/s) but summed in the same order into one
  // accumulator: the partials keep their bits (the clip factor, and with it the training trajectory,
  // is sensitive to the norm's last bits -- profiles/r04_norm)
  float s = 0.f;
  const size_t nv = n >> 3, stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    float x[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_g8(g, i + u * stride, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[u][j] * x[u][j];
  }
  for (; i < nv; i += stride) {
    float x[8];
    load_g8(g, i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * x[j];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

void adamw_step(at::Tensor& master, at::Tensor& m, at::Tensor& v, const at::Tensor& g, at::Tensor& w, const at::Tensor& hp) {
  CHECK_F32(master);
  CHECK_F32(m);
  CHECK_F32(v);
  CHECK_GRAD(g);
  CHECK_BF16(w);
  CHECK_F32(hp);
  const size_t n = master.numel();
  TORCH_CHECK(n % 8 == 0 && (size_t)m.numel() == n && (size_t)v.numel() == n && (size_t)g.numel() == n && (size_t)w.numel() == n,
              "adamw: flat buffers must have equal sizes, a multiple of 8");
  TORCH_CHECK(hp.numel() >= 8, "adamw: hp needs 8 entries");
  if (!n) return;
  if (g.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(adamw_kernel<float>, dim3(grid_for(n / 8)), dim3(256), 0, cur_stream(), master.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr<float>(), bpm(w), hp.data_ptr<float>(), n);
  else
    hipLaunchKernelGGL(adamw_kernel<u16>, dim3(grid_for(n / 8)), dim3(256), 0, cur_stream(), master.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), bp(g), bpm(w), hp.data_ptr<float>(), n);
}

// sqnorm + (optionally) the step counter: block 0 / thread 0 adds 1 to ``tick`` — nothing else in
// this kernel reads it; the AdamW kernel after it in stream order does.
template <typename G>
__global__ __launch_bounds__(256) void sqnorm_tick_kernel(const G* __restrict__ g, float* __restrict__ part, size_t n,
                                                          float* __restrict__ tick) {
  __shared__ float red[4];
  float s = 0.f;
  const size_t nv = n >> 3;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
    float x[8];
    load_g8(g, i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * x[j];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    if (tick != nullptr && blockIdx.x == 0) tick[0] = tick[0] + 1.f;
  }
}

// ============================================================================ synthetic MNIST
// One block per image: label = hash(seed, step, image) % classes, pixel = (prototype[label] +
// noise * N(0,1) - mean) / std in bf16, N(0,1) by Box-Muller from a counter-based hash of
// (seed, step, pixel index).  ``step`` is read from the device (the optimizer's step counter), so a
// captured graph draws a fresh batch every replay with no host involvement.  Reference:
// ``models/mnist.py synth_reference`` (same hash in numpy).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return mix32(a ^ mix32(b ^ mix32(c))); }

__global__ __launch_bounds__(256) void mnist_synth_kernel(const float* __restrict__ proto, u16* __restrict__ x,
                                                          int64_t* __restrict__ y, const float* __restrict__ tptr, uint32_t seed,
                                                          int classes, int pixels, float noise, float mean, float inv_std) {
  const int b = blockIdx.x;
  const uint32_t step = (uint32_t)tptr[0];
  const uint32_t lab = hash3(seed, step, 0x9e3779b9U ^ (uint32_t)b) % (uint32_t)classes;
  if (threadIdx.x == 0) y[b] = (int64_t)lab;
  const float* pr = proto + (size_t)lab * pixels;
  u16* xo = x + (size_t)b * pixels;
  for (int p = threadIdx.x * 2; p < pixels; p += 512) {
    const uint32_t h1 = hash3(seed ^ 0x85ebca6bU, step, (uint32_t)b * (uint32_t)pixels + (uint32_t)p);
    const uint32_t h2 = mix32(h1 ^ 0x27d4eb2fU);
    const float u1 = (float)((h1 >> 8) + 1u) * (1.f / 16777216.f);  // (0, 1]
    const float u2 = (float)(h2 >> 8) * (1.f / 16777216.f);         // [0, 1)
    const float r = sqrtf(-2.f * logf(u1));
    const float a = 6.28318530718f * u2;
    xo[p] = f2bf((pr[p] + noise * r * cosf(a) - mean) * inv_std);
    if (p + 1 < pixels) xo[p + 1] = f2bf((pr[p + 1] + noise * r * sinf(a) - mean) * inv_std);
  }
}

std::vector<at::Tensor> mnist_synth(const at::Tensor& proto, int64_t batch, const at::Tensor& step, int64_t seed, double noise,
                                    double mean, double std_) {
  CHECK_F32(proto);
  CHECK_F32(step);
  TORCH_CHECK(proto.dim() == 4 && proto.size(1) == 1, "prototypes must be [classes, 1, H, W]");
  TORCH_CHECK(batch > 0 && batch < (1 << 24), "batch out of range");
  const int classes = (int)proto.size(0), H = (int)proto.size(2), W = (int)proto.size(3), pixels = H * W;
  auto x = at::empty({batch, 1, H, W}, proto.options().dtype(at::kBFloat16));
  auto y = at::empty({batch}, proto.options().dtype(at::kLong));
  hipLaunchKernelGGL(mnist_synth_kernel, dim3((unsigned)batch), dim3(256), 0, cur_stream(), proto.data_ptr<float>(), bpm(x),
                     y.data_ptr<int64_t>(), step.data_ptr<float>(), (uint32_t)seed, classes, pixels, (float)noise, (float)mean,
                     (float)(1.0 / std_));
  return {x, y};
}

at::Tensor sq_norm_parts(const at::Tensor& g, c10::optional<at::Tensor> tick) {
  CHECK_GRAD(g);
  const size_t n = g.numel();
  TORCH_CHECK(n % 8 == 0, "sq_norm_parts: size must be a multiple of 8");
  float* tk = nullptr;
  if (tick.has_value()) {
    CHECK_F32(*tick);
    tk = tick->data_ptr<float>();
  }
  const int grid = (int)std::max<size_t>(1, std::min<size_t>((n / 8 + 255) / 256, 1024));
  auto part = at::empty({grid}, g.options().dtype(at::kFloat));  // every slot written
  if (g.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(sqnorm_tick_kernel<float>, dim3(grid), dim3(256), 0, cur_stream(), g.data_ptr<float>(), part.data_ptr<float>(), n,
                       tk);
  else
    hipLaunchKernelGGL(sqnorm_tick_kernel<u16>, dim3(grid), dim3(256), 0, cur_stream(), bp(g), part.data_ptr<float>(), n, tk);
  return part;
}

void adamw_step_dev(at::Tensor& master, at::Tensor& m, at::Tensor& v, const at::Tensor& g, at::Tensor& w, const at::Tensor& hp,
                    c10::optional<at::Tensor> part, const at::Tensor& t) {
  CHECK_F32(master);
  CHECK_F32(m);
  CHECK_F32(v);
  CHECK_GRAD(g);
  CHECK_BF16(w);
  CHECK_F32(hp);
  CHECK_F32(t);
  const size_t n = master.numel();
  TORCH_CHECK(n % 8 == 0 && (size_t)m.numel() == n && (size_t)v.numel() == n && (size_t)g.numel() == n && (size_t)w.numel() == n,
              "adamw: flat buffers must have equal sizes, a multiple of 8");
  TORCH_CHECK(hp.numel() >= 7, "adamw_step_dev: hp needs 7 entries");
  const float* pp = nullptr;
  int np = 0;
  if (part.has_value()) {
    CHECK_F32(*part);
    pp = part->data_ptr<float>();
    np = (int)part->numel();
  }
  if (!n) return;
  if (g.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(adamw_dev_kernel<float>, dim3(grid_for(n / 8)), dim3(256), 0, cur_stream(), master.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr<float>(), bpm(w), hp.data_ptr<float>(), pp, np,
                       t.data_ptr<float>(), n);
  else
    hipLaunchKernelGGL(adamw_dev_kernel<u16>, dim3(grid_for(n / 8)), dim3(256), 0, cur_stream(), master.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), bp(g), bpm(w), hp.data_ptr<float>(), pp, np,
                       t.data_ptr<float>(), n);
}

at::Tensor sq_norm(const at::Tensor& g) {
  CHECK_GRAD(g);
  const size_t n = g.numel();
  TORCH_CHECK(n % 8 == 0, "sq_norm: size must be a multiple of 8");
  const int grid = 1024;
  auto part = at::zeros({grid}, g.options().dtype(at::kFloat));
  if (n && g.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(sqnorm_kernel<float>, dim3(grid), dim3(256), 0, cur_stream(), g.data_ptr<float>(), part.data_ptr<float>(), n);
  else if (n)
    hipLaunchKernelGGL(sqnorm_kernel<u16>, dim3(grid), dim3(256), 0, cur_stream(), bp(g), part.data_ptr<float>(), n);
  return part.sum();
}

}  // namespace

namespace gtk_mnist {  // csrc/ops/mnist_conv.hip
at::Tensor conv1_fwd(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1);
std::vector<at::Tensor> conv2_pool_fwd(const at::Tensor& h1, const at::Tensor& w2, const at::Tensor& b2, const at::Tensor& step,
                                       int64_t seed, double p_drop);
void conv_bwd(const at::Tensor& dp, const at::Tensor& code, const at::Tensor& x, const at::Tensor& h1, const at::Tensor& w1,
              const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& gw1, at::Tensor& gb1, at::Tensor& gw2,
              at::Tensor& gb2, double p_drop, bool accumulate);
std::vector<at::Tensor> relu_dropout_fwd(const at::Tensor& h, const at::Tensor& step, int64_t seed, double p_drop);
at::Tensor relu_dropout_bwd(const at::Tensor& dy, const at::Tensor& mask, at::Tensor& gb, double p_drop, bool accumulate);
std::vector<at::Tensor> xent10_fwd(const at::Tensor& logits, const at::Tensor& labels);
at::Tensor xent10_bwd(const at::Tensor& dlog, const at::Tensor& g, at::Tensor& gb, bool accumulate);
}  // namespace gtk_mnist

namespace gtk_attn {  // csrc/ops/attention.hip
std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale);
std::vector<at::Tensor> attn_fwd_t(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale);
std::vector<at::Tensor> attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                 const at::Tensor& out, const at::Tensor& lse, double scale);
}  // namespace gtk_attn

namespace gtk_xpose {  // csrc/ops/transpose.hip
at::Tensor transpose_bf16(const at::Tensor& x);
void transpose_bf16_out(const at::Tensor& x, at::Tensor& y);
}  // namespace gtk_xpose

namespace gtk_shadow {  // csrc/ops/comm_shadow.hip
void comm_shadow(const at::Tensor& src, at::Tensor& dst, int64_t bytes, int64_t ctas, double micros);
}  // namespace gtk_shadow

namespace gtk_adamw {  // csrc/ops/adamw_t.hip
void adamw_step_t(at::Tensor& master, at::Tensor& m, at::Tensor& v, const at::Tensor& g, at::Tensor& w, at::Tensor& wt,
                  const at::Tensor& hp, const at::Tensor& mats, int64_t total_tiles, const at::Tensor& ranges,
                  int64_t max_range, c10::optional<at::Tensor> part, c10::optional<at::Tensor> t, int64_t ahead);
}  // namespace gtk_adamw

PYBIND11_MODULE(_fused, m) {
  m.def("attn_fwd", &gtk_attn::attn_fwd, "causal GQA flash attention forward (bf16, D=128): -> (o [B,S,H,D], lse2 [B,H,S])");
  m.def("attn_fwd_t", &gtk_attn::attn_fwd_t, "attn_fwd that also writes O^T [H*D, B*S]: -> (o, lse2, ot)");
  m.def("attn_bwd", &gtk_attn::attn_bwd, "flash attention backward: -> (dq, dk, dv)");
  m.doc() = "gfx950 fused kernels for the Llama-3 DP validation workload";
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.def("add_rmsnorm_bwd", &add_rmsnorm_bwd);
  m.def("embed_bwd_into", &embed_bwd_into, "embedding gradient rows summed per token (sorted positions) into a zeroed [V, D] bf16 view");
  m.def("rmsnorm_bwd_into", &rmsnorm_bwd_into, "rmsnorm_bwd writing dW into a given bf16 view; returns dx");
  m.def("add_rmsnorm_bwd_into", &add_rmsnorm_bwd_into, "add_rmsnorm_bwd writing dW into a given bf16 view; returns dx");
  m.def("rope_split_fwd", &rope_split_fwd);
  m.def("rope_split_bwd", &rope_split_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("swiglu_bwd_t128", &swiglu_bwd_t128, "swiglu_bwd_t with 64 x 128 tiles (bit-identical)");
  m.def("swiglu_fwd_t128", &swiglu_fwd_t128, "swiglu_fwd_t with 64 x 128 tiles; T multiple of 64, F of 128");
  m.def("swiglu_fwd_t", &swiglu_fwd_t, "swiglu forward -> (h [T, F], h^T [F, T]); T, F multiples of 64");
  m.def("swiglu_bwd_t", &swiglu_bwd_t, "swiglu backward -> (dgu [T, 2F], dgu^T [2F, T]); T, F multiples of 64");
  m.def("xent_fwd", &xent_fwd);
  m.def("rope_split_bwd_t", &rope_split_bwd_t, "rope_split_bwd that also returns dqkv^T; head dim 128, S multiple of 64");
  m.def("xent_bwd_inplace", &xent_bwd_inplace);
  m.def("xent_bwd_t", &xent_bwd_t, "xent_bwd_inplace that also returns dlogits^T [V, T]; T multiple of 64, V of 128");
  m.def("adamw_step", &adamw_step);
  m.def("sq_norm", &sq_norm);
  m.def("sq_norm_parts", &sq_norm_parts, "sum-of-squares partials of a bf16 buffer; optionally advance a step counter");
  m.def("adamw_step_dev", &adamw_step_dev, "AdamW with device-side bias correction and clipping (graph-capturable)");
  m.def("mnist_synth", &mnist_synth, "synthetic MNIST batch on the device, indexed by a device step counter");
  m.def("mnist_conv1_fwd", &gtk_mnist::conv1_fwd, "MNIST conv1 + ReLU, NHWC bf16");
  m.def("mnist_conv2_pool_fwd", &gtk_mnist::conv2_pool_fwd, "MNIST conv2 + ReLU + 2x2 max-pool + dropout (MFMA)");
  m.def("mnist_conv_bwd", &gtk_mnist::conv_bwd, "MNIST conv stack backward into the flat gradient (MFMA)");
  m.def("mnist_relu_dropout_fwd", &gtk_mnist::relu_dropout_fwd, "ReLU + hash dropout, keep mask");
  m.def("mnist_relu_dropout_bwd", &gtk_mnist::relu_dropout_bwd, "ReLU/dropout backward + bias gradient");
  m.def("mnist_xent10_fwd", &gtk_mnist::xent10_fwd, "10-class softmax cross-entropy: mean loss + unscaled gradient");
  m.def("mnist_xent10_bwd", &gtk_mnist::xent10_bwd, "scaled logits gradient + bias gradient");
  m.def("transpose_bf16", &gtk_xpose::transpose_bf16, "contiguous [R, C] bf16 -> [C, R] (R, C multiples of 64)");
  m.def("transpose_bf16_out", &gtk_xpose::transpose_bf16_out, "transpose [R, C] bf16 into a contiguous [C, R] buffer");
  m.def("comm_shadow", &gtk_shadow::comm_shadow,
        "shadow of a DP collective: `ctas` workgroups copy `bytes` src -> dst, paced over at least `micros` us");
  m.def("adamw_step_t", &gtk_adamw::adamw_step_t,
        "AdamW over the flat buffers that also writes W^T of the listed matrices (tile kernel) and updates the listed "
        "ranges (flat kernel); part/t given = the device-side (graph-capturable) hyper-parameter form");
}
