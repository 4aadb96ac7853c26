// MNIST CNN convolution stack on gfx950 (models/mnist.py, the Gaia paper's Exp. 6 workload).
//
// conv1 (1->32, 3x3) + ReLU, conv2 (32->64, 3x3) + ReLU + 2x2 max-pool + dropout, and their backward,
// as five launches instead of MIOpen's ~45 (layout transposes, casts, bias reductions, naive conv1):
//
//   conv1_fwd        FMA, one thread per (pixel, 8 channels); writes h1 NHWC bf16
//   conv2_pool_fwd   MFMA implicit GEMM, M = output pixels ordered so that a lane's four accumulator
//                    rows are one 2x2 pooling window (pool = max over the lane's registers, no
//                    shuffles); epilogue adds bias, ReLU, pools, applies dropout from a counter-based
//                    hash, writes the pooled map and one code byte per element (argmax | pos | keep)
//   conv2_dgrad      MFMA implicit GEMM over the 9 taps x 64 output channels; dy2 is never stored: the
//                    A fragment is rebuilt from the pooled gradient and the code bytes; the epilogue
//                    applies conv1's ReLU mask and accumulates conv1's weight/bias gradient in
//                    registers (dz1 is never stored either) -> per-workgroup partials
//   conv2_wgrad      MFMA, M = 64 output channels, N = 9 taps x 32 input channels, K = output pixels
//                    of one row (24, padded to 32); dy2 and three column-shifted copies of the h1 rows
//                    are staged transposed in LDS so every fragment is one 16-byte LDS read
//   conv_grad_reduce sums the partials in a fixed order (deterministic) into the flat bf16 gradient
//
// Layouts (bf16): x [B,28,28]; h1 [B,26,26,32]; pooled p [B,12,12,64] (== fc1's NHWC input order);
// conv1.w [32][3][3] (+ bias [32]); conv2.w [64][3][3][32] (co, ky, kx, ci) (+ bias [64]).
// MFMA: v_mfma_f32_16x16x32_bf16 — lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], and
// C/D col = l&15, row = 4(l>>4) + reg (cdna_hip_programming.md "Fragment layout").
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>

namespace gtk_mnist {
namespace {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IMG = 28, H1 = 26, C1 = 32, H2 = 24, C2 = 64, HP = 12;
constexpr int WIN_PER_IMG = HP * HP;      // 144 pooling windows
constexpr int PIX1 = H1 * H1;             // 676 conv1 output pixels
constexpr int KW2 = 9 * C1;               // 288 = conv2 reduction length
constexpr int NW2 = C2 * KW2;             // 18432 conv2 weights
constexpr int P2 = NW2 + C2;              // conv2 partial row: weights + bias
constexpr int P1 = C1 * 10;               // conv1 partial row: [ci][9 taps + bias]

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return mix32(a ^ mix32(b ^ mix32(c))); }

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }
const u16* bp(const at::Tensor& t) { return reinterpret_cast<const u16*>(t.data_ptr()); }
u16* bpm(at::Tensor& t) { return reinterpret_cast<u16*>(t.data_ptr()); }

// ------------------------------------------------------------------------------- conv1 forward
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ w1,
                                                        const u16* __restrict__ b1, u16* __restrict__ h1, int npix) {
  const int tid = blockIdx.x * 256 + threadIdx.x;
  if (tid >= npix * 4) return;
  const int cg = tid & 3, pix = tid >> 2;
  const int b = pix / PIX1, rem = pix - b * PIX1, y = rem / H1, xx = rem - y * H1;
  const u16* xi = x + (size_t)b * IMG * IMG + y * IMG + xx;
  float in[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) in[t] = bf2f(xi[(t / 3) * IMG + t % 3]);
  u16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    float s = bf2f(b1[c]);
#pragma unroll
    for (int t = 0; t < 9; ++t) s += bf2f(w1[c * 9 + t]) * in[t];
    out[j] = f2bf(fmaxf(s, 0.f));
  }
  reinterpret_cast<u16x8*>(h1)[(size_t)pix * 4 + cg] = out;
}

// ------------------------------------------------------------------- conv2 + pool forward (MFMA)
constexpr int W2S = KW2 + 8;  // LDS row stride of conv2.w per output channel (pad: spreads banks)

__global__ __launch_bounds__(256) void conv2_pool_fwd_kernel(const u16* __restrict__ h1, const u16* __restrict__ w2,
                                                             const u16* __restrict__ b2, u16* __restrict__ p,
                                                             uint8_t* __restrict__ code, const float* __restrict__ tptr,
                                                             uint32_t seed, uint32_t drop_thresh, float keep_scale, int nwin) {
  __shared__ __attribute__((aligned(16))) u16 ws[C2 * W2S];
  for (int i = threadIdx.x; i < C2 * (KW2 / 8); i += 256) {
    const int co = i / (KW2 / 8), ch = i - co * (KW2 / 8);
    *reinterpret_cast<u16x8*>(&ws[co * W2S + ch * 8]) = reinterpret_cast<const u16x8*>(w2)[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
  const int wbase = (blockIdx.x * 4 + wave) * 8;  // 2 m-tiles x 4 windows per wave
  const uint32_t step = (uint32_t)tptr[0];
  int abase[2];
  bool aval[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    int win = wbase + mt * 4 + (r >> 2);
    aval[mt] = win < nwin;
    if (!aval[mt]) win = 0;
    const int q = r & 3, b = win / WIN_PER_IMG, pw = win - b * WIN_PER_IMG, py = pw / HP, px = pw - py * HP;
    const int y = 2 * py + (q >> 1), xx = 2 * px + (q & 1);
    abase[mt] = ((b * H1 + y) * H1 + xx) * C1 + h * 8;
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int toff = ((t / 3) * H1 + t % 3) * C1;
    bf16x8 a[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (aval[mt]) v = *reinterpret_cast<const u16x8*>(h1 + abase[mt] + toff);
      a[mt] = as_bf(v);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16x8 bf = as_bf(*reinterpret_cast<const u16x8*>(&ws[(nt * 16 + r) * W2S + t * C1 + h * 8]));
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt][nt] = mfma16(a[mt], bf, acc[mt][nt]);
    }
  }
  // lane: window wbase + 4mt + h (rows 4h..4h+3 = its 4 pixels), channel nt*16 + r
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int win = wbase + mt * 4 + h;
    if (win >= nwin) continue;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int co = nt * 16 + r;
      float m = acc[mt][nt][0];
      int am = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (acc[mt][nt][q] > m) m = acc[mt][nt][q], am = q;
      m += bf2f(b2[co]);
      const bool pos = m > 0.f;
      const bool keep = (hash3(seed, step, (uint32_t)(win * C2 + co)) >> 8) >= drop_thresh;
      const size_t o = (size_t)win * C2 + co;
      p[o] = f2bf(pos && keep ? m * keep_scale : 0.f);
      code[o] = (uint8_t)(am | (pos ? 4 : 0) | (keep ? 8 : 0));
    }
  }
}

// dy2 fragment: 8 channels co0..co0+7 of conv2's output pixel (y, x) from the pooled gradient.
__device__ __forceinline__ void dy2_frag(const u16* __restrict__ dp, const uint8_t* __restrict__ code, int b, int y, int xx,
                                         int co0, float dscale, float* v) {
  const int win = (b * HP + (y >> 1)) * HP + (xx >> 1), q = (y & 1) * 2 + (xx & 1);
  const uint64_t c8 = *reinterpret_cast<const uint64_t*>(code + (size_t)win * C2 + co0);
  const u16x8 d8 = *reinterpret_cast<const u16x8*>(dp + (size_t)win * C2 + co0);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t c = (uint32_t)(c8 >> (8 * j)) & 0xffu;
    v[j] = ((c & 3u) == (uint32_t)q && (c & 12u) == 12u) ? bf2f(d8[j]) * dscale : 0.f;
  }
}

// ------------------------------------------------------ conv2 dgrad + conv1 wgrad partials (MFMA)
constexpr int WTS = C2 + 8;   // LDS row stride of the transposed conv2.w: [tap][ci][co]
constexpr int DG_ROWS = 4;    // input rows of h1 per workgroup (one per wave)
constexpr int DYW = 34;       // dy2 tile columns: x = -2 .. 31 (zero outside 0..23)
constexpr int DYC = C2 + 8;   // dy2 tile channel stride (pad)

// Workgroup = (image b, input rows 4g .. 4g+3); wave w owns input row 4g + w, as two 16-pixel m-tiles
// (x = 0..31, 26 valid).  The dy2 rows it needs (4g-2 .. 4g+3) are rebuilt once from the pooled
// gradient and code bytes into a zero-bordered LDS tile, so every A fragment is one 16-byte LDS read.
__global__ __launch_bounds__(256) void conv2_dgrad_kernel(const u16* __restrict__ dp, const uint8_t* __restrict__ code,
                                                          const u16* __restrict__ w2, const u16* __restrict__ h1,
                                                          const u16* __restrict__ x, float* __restrict__ part1, float dscale) {
  __shared__ __attribute__((aligned(16))) u16 wt[9 * C1 * WTS];
  __shared__ __attribute__((aligned(16))) u16 dyl[(DG_ROWS + 2) * DYW * DYC];
  __shared__ float red[4][P1];
  constexpr int GROUPS = (H1 + DG_ROWS - 1) / DG_ROWS;  // 7
  const int b = blockIdx.x / GROUPS, yi0 = (blockIdx.x - b * GROUPS) * DG_ROWS;
  for (int i = threadIdx.x; i < C2 * (KW2 / 8); i += 256) {
    const int co = i / (KW2 / 8), ch = i - co * (KW2 / 8), tap = ch >> 2, ci0 = (ch & 3) * 8;
    const u16x8 v = reinterpret_cast<const u16x8*>(w2)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) wt[(tap * C1 + ci0 + j) * WTS + co] = v[j];
  }
  for (int i = threadIdx.x; i < (DG_ROWS + 2) * DYW * 8; i += 256) {
    const int ry = i / (DYW * 8), rem = i - ry * (DYW * 8), xs = rem >> 3, co0 = (rem & 7) * 8;
    const int y = yi0 - 2 + ry, xx = xs - 2;
    u16x8 u = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (y >= 0 && y < H2 && xx >= 0 && xx < H2) {
      float v[8];
      dy2_frag(dp, code, b, y, xx, co0, dscale, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = f2bf(v[j]);
    }
    *reinterpret_cast<u16x8*>(&dyl[(ry * DYW + xs) * DYC + co0]) = u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
  const int yi = yi0 + wave;
  f32x4 acc[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ky = t / 3, kx = t % 3;
    const int arow = (wave - ky + 2) * DYW;  // dy2 row yi - ky
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const int co0 = kc * 32 + h * 8;
      bf16x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)  // dy2 column xi - kx, tile column xi - kx + 2 <= 33
        a[mt] = as_bf(*reinterpret_cast<const u16x8*>(&dyl[(arow + mt * 16 + r - kx + 2) * DYC + co0]));
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bf16x8 bf = as_bf(*reinterpret_cast<const u16x8*>(&wt[(t * C1 + nt * 16 + r) * WTS + co0]));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt][nt] = mfma16(a[mt], bf, acc[mt][nt]);
      }
    }
  }
  // lane: channel ci = nt*16 + r, pixels (yi, x = 16mt + 4h + reg)
  float w1acc[2][10];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int t = 0; t < 10; ++t) w1acc[nt][t] = 0.f;
  if (yi < H1) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int xi = mt * 16 + 4 * h + reg;
        if (xi >= H1) continue;
        const u16* xp = x + (size_t)b * IMG * IMG + yi * IMG + xi;
        float xin[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) xin[t] = bf2f(xp[(t / 3) * IMG + t % 3]);
        const size_t gp = ((size_t)b * H1 + yi) * H1 + xi;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float dz = bf2f(h1[gp * C1 + nt * 16 + r]) > 0.f ? acc[mt][nt][reg] : 0.f;
#pragma unroll
          for (int t = 0; t < 9; ++t) w1acc[nt][t] += dz * xin[t];
          w1acc[nt][9] += dz;
        }
      }
    }
  }
  // lanes r, r+16, r+32, r+48 share a channel: fold the lane quarters, then the waves through LDS
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      float v = w1acc[nt][t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (h == 0) red[wave][(nt * 16 + r) * 10 + t] = v;
    }
  __syncthreads();
  for (int i = threadIdx.x; i < P1; i += 256)
    part1[(size_t)blockIdx.x * P1 + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// ------------------------------------------------------------------- conv2 wgrad partials (MFMA)
constexpr int DYS = 40;  // LDS row stride (elements) of dy2^T rows (32 pixels + pad)
constexpr int HTS = 40;  // ... of the shifted h1^T rows
constexpr int HCHUNKS = 3 * H1 * 4;  // 312 16-byte chunks of h1 per output row (rows y..y+2)

// Workgroup = a run of consecutive output rows (b, y); per row, K = 24 pixels (padded to 32).  The
// next row's code bytes, pooled gradient and h1 chunks are loaded into registers while the MFMAs of
// the current row run, then written transposed into LDS.
__global__ __launch_bounds__(256) void conv2_wgrad_kernel(const u16* __restrict__ dp, const uint8_t* __restrict__ code,
                                                          const u16* __restrict__ h1, float* __restrict__ part2, float dscale,
                                                          int nrows, int rows_per_wg) {
  __shared__ __attribute__((aligned(16))) u16 dyT[C2 * DYS];          // [co][x]
  __shared__ __attribute__((aligned(16))) u16 hT[9 * C1 * HTS];       // [ky][shift][ci][x]
  __shared__ float dbp[192][9];
  for (int i = threadIdx.x; i < C2 * DYS; i += 256) dyT[i] = 0;
  for (int i = threadIdx.x; i < 9 * C1 * HTS; i += 256) hT[i] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
  f32x4 acc[18];
#pragma unroll
  for (int n = 0; n < 18; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int row0 = blockIdx.x * rows_per_wg, row1 = min(nrows, row0 + rows_per_wg);
  // this thread's staging tasks: one dy2 (x, 8-channel chunk) if < 192; h1 chunks tid and tid + 256
  const int dx = threadIdx.x >> 3, dco0 = (threadIdx.x & 7) * 8;
  uint64_t c8 = 0;
  u16x8 d8 = u16x8{0, 0, 0, 0, 0, 0, 0, 0}, hv0 = d8, hv1 = d8;
  auto load_row = [&](int gr) {
    const int b = gr / H2, y = gr - b * H2;
    if (threadIdx.x < 192) {
      const int win = (b * HP + (y >> 1)) * HP + (dx >> 1);
      c8 = *reinterpret_cast<const uint64_t*>(code + (size_t)win * C2 + dco0);
      d8 = *reinterpret_cast<const u16x8*>(dp + (size_t)win * C2 + dco0);
    }
    const size_t base = ((size_t)b * H1 + y) * H1 * C1;  // h1 row y of image b; chunk i -> (ky, x, ci0)
    hv0 = *reinterpret_cast<const u16x8*>(h1 + base + (size_t)threadIdx.x * 8);
    if (threadIdx.x + 256 < HCHUNKS) hv1 = *reinterpret_cast<const u16x8*>(h1 + base + (size_t)(threadIdx.x + 256) * 8);
  };
  auto store_h = [&](int i, const u16x8& v) {
    const int ky = i / (H1 * 4), rem = i - ky * (H1 * 4), xx = rem >> 2, ci0 = (rem & 3) * 8;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int xd = xx - s;
      if (xd >= 0 && xd < 32) {
#pragma unroll
        for (int j = 0; j < 8; ++j) hT[((ky * 3 + s) * C1 + ci0 + j) * HTS + xd] = v[j];
      }
    }
  };
  if (row0 < row1) load_row(row0);
  __syncthreads();
  for (int gr = row0; gr < row1; ++gr) {
    const int y = gr - (gr / H2) * H2;
    if (threadIdx.x < 192) {  // dy2 row, written transposed
      const int q = (y & 1) * 2 + (dx & 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t c = (uint32_t)(c8 >> (8 * j)) & 0xffu;
        const float v = ((c & 3u) == (uint32_t)q && (c & 12u) == 12u) ? bf2f(d8[j]) * dscale : 0.f;
        db[j] += v;
        dyT[(dco0 + j) * DYS + dx] = f2bf(v);
      }
    }
    store_h(threadIdx.x, hv0);
    if (threadIdx.x + 256 < HCHUNKS) store_h(threadIdx.x + 256, hv1);
    __syncthreads();
    if (gr + 1 < row1) load_row(gr + 1);  // in flight during the MFMAs below
    const bf16x8 a = as_bf(*reinterpret_cast<const u16x8*>(&dyT[(wave * 16 + r) * DYS + h * 8]));
#pragma unroll
    for (int n = 0; n < 18; ++n) {
      const bf16x8 bf = as_bf(*reinterpret_cast<const u16x8*>(&hT[((n >> 1) * C1 + (n & 1) * 16 + r) * HTS + h * 8]));
      acc[n] = mfma16(a, bf, acc[n]);
    }
    __syncthreads();
  }
  float* out = part2 + (size_t)blockIdx.x * P2;
#pragma unroll
  for (int n = 0; n < 18; ++n)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      out[(wave * 16 + 4 * h + reg) * KW2 + (n >> 1) * C1 + (n & 1) * 16 + r] = acc[n][reg];
  if (threadIdx.x < 192)
#pragma unroll
    for (int j = 0; j < 8; ++j) dbp[threadIdx.x][j] = db[j];
  __syncthreads();
  if (threadIdx.x < C2) {
    const int chunk = threadIdx.x >> 3, j = threadIdx.x & 7;
    float s = 0.f;
    for (int xx = 0; xx < H2; ++xx) s += dbp[xx * 8 + chunk][j];
    out[NW2 + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------ partials -> gradient
// Block = 64 gradient columns x 4 partial slices (coalesced 256-B rows); slice s sums partials
// s, s+4, ... and the slices are added in a fixed order: deterministic.
__global__ __launch_bounds__(256) void conv_grad_reduce_kernel(const float* __restrict__ part1, int n1,
                                                               const float* __restrict__ part2, int n2, u16* __restrict__ gw1,
                                                               u16* __restrict__ gb1, u16* __restrict__ gw2,
                                                               u16* __restrict__ gb2, int accumulate) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;  // P2 = 289 x 64 and P1 = 5 x 64: no block straddles the two
  const bool second = col >= P2;
  const float* src = second ? part1 + (col - P2) : part2 + col;
  const int n = second ? n1 : n2;
  const size_t stride = second ? P1 : P2;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < P2 + P1) {
    int k = sl;
    for (; k + 12 < n; k += 16) {
      s0 += src[(size_t)k * stride];
      s1 += src[(size_t)(k + 4) * stride];
      s2 += src[(size_t)(k + 8) * stride];
      s3 += src[(size_t)(k + 12) * stride];
    }
    for (; k < n; k += 4) s0 += src[(size_t)k * stride];
  }
  red[sl][c] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sl != 0 || col >= P2 + P1) return;
  float s = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  u16* dst;
  if (!second) {
    dst = col < NW2 ? gw2 + col : gb2 + (col - NW2);
  } else {
    const int j = col - P2, ci = j / 10, t = j - ci * 10;
    dst = t < 9 ? gw1 + ci * 9 + t : gb1 + ci;
  }
  if (accumulate) s += bf2f(*dst);
  *dst = f2bf(s);
}

#define CHECK_BF16(t) TORCH_CHECK((t).is_cuda() && (t).scalar_type() == at::kBFloat16 && (t).is_contiguous(), #t " must be a contiguous bf16 GPU tensor")

void check_w(const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2) {
  CHECK_BF16(w1);
  CHECK_BF16(b1);
  CHECK_BF16(w2);
  CHECK_BF16(b2);
  TORCH_CHECK(w1.numel() == C1 * 9 && b1.numel() == C1 && w2.numel() == NW2 && b2.numel() == C2,
              "mnist conv: weights must be conv1 [32,3,3,1], conv2 [64,3,3,32] (+ biases)");
}

uint32_t drop_threshold(double p) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout probability must be in [0, 1)");
  return (uint32_t)(p * 16777216.0 + 0.5);  // keep iff hash >> 8 >= threshold
}

}  // namespace

at::Tensor conv1_fwd(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1) {
  CHECK_BF16(x);
  CHECK_BF16(w1);
  CHECK_BF16(b1);
  TORCH_CHECK(x.numel() % (IMG * IMG) == 0 && x.size(-1) == IMG && x.size(-2) == IMG, "x must be [B,1,28,28]");
  TORCH_CHECK(w1.numel() == C1 * 9 && b1.numel() == C1, "conv1 weights must be [32,3,3,1] + [32]");
  const int64_t B = x.numel() / (IMG * IMG);
  TORCH_CHECK(B > 0 && B * PIX1 * 4 < (1LL << 31), "batch out of range");
  auto h1 = at::empty({B, H1, H1, C1}, x.options());
  const int npix = (int)(B * PIX1);
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3((npix * 4 + 255) / 256), dim3(256), 0, cur_stream(), bp(x), bp(w1), bp(b1),
                     bpm(h1), npix);
  return h1;
}

std::vector<at::Tensor> conv2_pool_fwd(const at::Tensor& h1, const at::Tensor& w2, const at::Tensor& b2, const at::Tensor& step,
                                       int64_t seed, double p_drop) {
  CHECK_BF16(h1);
  CHECK_BF16(w2);
  CHECK_BF16(b2);
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kFloat && step.numel() >= 1, "step must be a fp32 GPU tensor");
  TORCH_CHECK(h1.dim() == 4 && h1.size(1) == H1 && h1.size(2) == H1 && h1.size(3) == C1, "h1 must be [B,26,26,32]");
  TORCH_CHECK(w2.numel() == NW2 && b2.numel() == C2, "conv2 weights must be [64,3,3,32] + [64]");
  const int64_t B = h1.size(0);
  TORCH_CHECK(B > 0 && B * WIN_PER_IMG * C2 < (1LL << 31), "batch out of range");
  auto p = at::empty({B, HP, HP, C2}, h1.options());
  auto code = at::empty({B, HP, HP, C2}, h1.options().dtype(at::kByte));
  const int nwin = (int)(B * WIN_PER_IMG);
  const float keep_scale = (float)(1.0 / (1.0 - p_drop));
  hipLaunchKernelGGL(conv2_pool_fwd_kernel, dim3((nwin + 31) / 32), dim3(256), 0, cur_stream(), bp(h1), bp(w2), bp(b2), bpm(p),
                     code.data_ptr<uint8_t>(), step.data_ptr<float>(), (uint32_t)seed, drop_threshold(p_drop), keep_scale, nwin);
  return {p, code};
}

void conv_bwd(const at::Tensor& dp, const at::Tensor& code, const at::Tensor& x, const at::Tensor& h1, const at::Tensor& w1,
              const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& gw1, at::Tensor& gb1, at::Tensor& gw2,
              at::Tensor& gb2, double p_drop, bool accumulate) {
  CHECK_BF16(dp);
  CHECK_BF16(x);
  CHECK_BF16(h1);
  check_w(w1, b1, w2, b2);
  check_w(gw1, gb1, gw2, gb2);
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kByte && code.is_contiguous(), "code must be uint8");
  const int64_t B = h1.size(0);
  TORCH_CHECK(h1.dim() == 4 && h1.size(1) == H1 && h1.size(2) == H1 && h1.size(3) == C1, "h1 must be [B,26,26,32]");
  TORCH_CHECK(dp.numel() == B * WIN_PER_IMG * C2 && code.numel() == B * WIN_PER_IMG * C2 && x.numel() == B * IMG * IMG,
              "dp/code/x sizes do not match the batch of h1");
  drop_threshold(p_drop);
  const float dscale = (float)(1.0 / (1.0 - p_drop));
  const int n1 = (int)(B * ((H1 + DG_ROWS - 1) / DG_ROWS));
  const int nrows = (int)(B * H2);
  const int n2 = (int)std::min<int64_t>(2 * B, 128);
  const int rows_per_wg = (nrows + n2 - 1) / n2;
  auto opts = dp.options().dtype(at::kFloat);
  auto part1 = at::empty({n1, P1}, opts);
  auto part2 = at::empty({n2, P2}, opts);
  hipStream_t st = cur_stream();
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(n1), dim3(256), 0, st, bp(dp), code.data_ptr<uint8_t>(), bp(w2), bp(h1), bp(x),
                     part1.data_ptr<float>(), dscale);
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(n2), dim3(256), 0, st, bp(dp), code.data_ptr<uint8_t>(), bp(h1),
                     part2.data_ptr<float>(), dscale, nrows, rows_per_wg);
  static_assert(P2 % 64 == 0 && P1 % 64 == 0, "reduce blocks must not straddle the two partial sets");
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3((P2 + P1) / 64), dim3(256), 0, st, part1.data_ptr<float>(), n1,
                     part2.data_ptr<float>(), n2, bpm(gw1), bpm(gb1), bpm(gw2), bpm(gb2), accumulate ? 1 : 0);
}

}  // namespace gtk_mnist
