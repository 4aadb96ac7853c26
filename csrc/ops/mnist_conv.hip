// MNIST CNN convolution stack on gfx950 (models/mnist.py, the Gaia paper's Exp. 6 workload).
//
// conv1 (1->32, 3x3) + ReLU, conv2 (32->64, 3x3) + ReLU + 2x2 max-pool + dropout, and their backward,
// as four launches instead of MIOpen's ~45 (layout transposes, casts, bias reductions, naive conv1):
//
//   conv1_fwd        FMA, one thread per (pixel, 8 channels); writes h1 NHWC bf16
//   conv2_pool_fwd   MFMA implicit GEMM, M = output pixels ordered so that a lane's four accumulator
//                    rows are one 2x2 pooling window (pool = max over the lane's registers, no
//                    shuffles); epilogue adds bias, ReLU, pools, applies dropout from a counter-based
//                    hash, writes the pooled map and one code byte per element (argmax | pos | keep)
//   conv2_bwd        one launch, two block roles running concurrently:
//   - dgrad          MFMA implicit GEMM over the 9 taps x 64 output channels; dy2 is never stored: the
//                    A fragment is rebuilt from the pooled gradient and the code bytes; the epilogue
//                    applies conv1's ReLU mask and accumulates conv1's weight/bias gradient in
//                    registers (dz1 is never stored either) -> per-workgroup partials
//   - wgrad          MFMA, M = 64 output channels, N = 9 taps x 32 input channels, K = output pixels
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
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

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

// 16x16x32 operand whose k index walks the ROWS of a row-major LDS image [k][cols] (ds_read_b64_tr_b16,
// cdna_hip_programming.md T10): lane l = 16g + 4q + p reads rows row0 + 8g + q (+4), columns
// col0 + 4p .. +3, and receives column col0 + (l & 15) for k = 8g .. 8g+7.  Whole-vector casts only
// (a per-element bit cast of a tr-read result miscompiles on this toolchain).  EXEC must be full.
__device__ __forceinline__ bf16x8 tr_frag16(const u16* img, int stride, int row0, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const u16* a = img + (row0 + 8 * g + q) * stride + col0 + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a + 4 * stride));
  return __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
}

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
// LDS row stride of conv2.w per output channel: 152 dwords makes the forward's ds_read_b128 B reads
// conflict-free (every 16-lane b128 group covers the 64 banks once; was 41 % conflict cycles at 148)
constexpr int W2S = KW2 + 16;

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
constexpr int DG_ROWS = 4;    // input rows of h1 per workgroup (one per wave)
// dy2 tile columns x = -2 .. 25 (zero outside 0..23).  Padded pixels x >= 26 of a wave's second
// m-tile read up to 6 columns past a row (into the next row, or past the tile into the h1 tile): finite
// values that only reach their own discarded output rows (MFMA rows are independent).
constexpr int DYW = 28;
constexpr int DYC = C2 + 16;  // 40 dwords: the A fragment's ds_read_b128 groups are conflict-free
constexpr int XROWS = DG_ROWS + 2;

// Workgroup = (image b, input rows 4g .. 4g+3); wave w owns input row 4g + w as two 16-pixel m-tiles
// (x = 0..31, 26 valid).  Everything the workgroup reads is staged once, with every global load
// issued before the first LDS write: conv2.w row-major (its k index, the output channel, walks rows:
// transposed reads give the B operand), the dy2 rows 4g-2 .. 4g+3 rebuilt from the pooled gradient
// and code bytes into a zero-bordered tile (A operand: one 16-byte read), and the h1 / x rows the
// epilogue needs for conv1's ReLU mask and weight gradient.
constexpr int DG_LDS_WS = C2 * W2S * 2, DG_LDS_DY = XROWS * DYW * DYC * 2, DG_LDS_H1 = DG_ROWS * H1 * C1 * 2,
              DG_LDS_X = (XROWS * IMG + 8) * 2;
constexpr int DG_LDS = DG_LDS_WS + DG_LDS_DY + DG_LDS_H1 + DG_LDS_X + 4 * P1 * 4;

__device__ __forceinline__ void conv2_dgrad_block(const u16* __restrict__ dp, const uint8_t* __restrict__ code,
                                                  const u16* __restrict__ w2, const u16* __restrict__ h1,
                                                  const u16* __restrict__ x, float* __restrict__ part1, float dscale, int blk,
                                                  char* smem) {
  u16* ws = reinterpret_cast<u16*>(smem);
  u16* dyl = reinterpret_cast<u16*>(smem + DG_LDS_WS);
  u16* h1t = reinterpret_cast<u16*>(smem + DG_LDS_WS + DG_LDS_DY);
  u16* xt = reinterpret_cast<u16*>(smem + DG_LDS_WS + DG_LDS_DY + DG_LDS_H1);
  float (*red)[P1] = reinterpret_cast<float (*)[P1]>(smem + DG_LDS_WS + DG_LDS_DY + DG_LDS_H1 + DG_LDS_X);
  constexpr int GROUPS = (H1 + DG_ROWS - 1) / DG_ROWS;  // 7
  const int b = blk / GROUPS, yi0 = (blk - b * GROUPS) * DG_ROWS;
  constexpr int WCH = C2 * (KW2 / 8) / 256;         // 9 conv2.w chunks per thread
  constexpr int DTASK = XROWS * DYW * 8;            // 1632 dy2 tasks
  constexpr int DPT = (DTASK + 255) / 256;          // 7 per thread
  constexpr int HTASK = DG_ROWS * H1 * 4;           // 416 h1 chunks
  const int nrows = min(DG_ROWS, H1 - yi0);
  u16x8 wv[WCH];
#pragma unroll
  for (int k = 0; k < WCH; ++k) wv[k] = reinterpret_cast<const u16x8*>(w2)[threadIdx.x + 256 * k];
  uint64_t cc[DPT];
  u16x8 dd[DPT];
#pragma unroll
  for (int k = 0; k < DPT; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int ry = i / (DYW * 8), rem = i - ry * (DYW * 8), xs = rem >> 3, co0 = (rem & 7) * 8;
    const int y = yi0 - 2 + ry, xx = xs - 2;
    cc[k] = 0;
    dd[k] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (i < DTASK && y >= 0 && y < H2 && xx >= 0 && xx < H2) {
      const size_t o = (size_t)((b * HP + (y >> 1)) * HP + (xx >> 1)) * C2 + co0;
      cc[k] = *reinterpret_cast<const uint64_t*>(code + o);
      dd[k] = *reinterpret_cast<const u16x8*>(dp + o);
    }
  }
  u16x8 hv[2];
  const u16* h1b = h1 + ((size_t)b * H1 + yi0) * H1 * C1;  // rows yi0 .. yi0+3 are contiguous
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + 256 * k;
    hv[k] = (i < HTASK && i < nrows * H1 * 4) ? reinterpret_cast<const u16x8*>(h1b)[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  uint32_t xv = 0;  // x rows yi0 .. yi0+5 (two bf16 per thread; rows past 27 are never read)
  const int xe = yi0 * IMG + 2 * threadIdx.x;
  if (threadIdx.x < XROWS * IMG / 2 && xe < IMG * IMG)
    xv = *reinterpret_cast<const uint32_t*>(x + (size_t)b * IMG * IMG + xe);
#pragma unroll
  for (int k = 0; k < WCH; ++k) {
    const int i = threadIdx.x + 256 * k, co = i / (KW2 / 8), ch = i - co * (KW2 / 8);
    *reinterpret_cast<u16x8*>(&ws[co * W2S + ch * 8]) = wv[k];
  }
#pragma unroll
  for (int k = 0; k < DPT; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i >= DTASK) break;
    const int ry = i / (DYW * 8), rem = i - ry * (DYW * 8), xs = rem >> 3, co0 = (rem & 7) * 8;
    const int y = yi0 - 2 + ry, xx = xs - 2, q = (y & 1) * 2 + (xx & 1);
    u16x8 u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t c = (uint32_t)(cc[k] >> (8 * j)) & 0xffu;  // 0 (never passes) outside the map
      u[j] = f2bf(((c & 3u) == (uint32_t)q && (c & 12u) == 12u) ? bf2f(dd[k][j]) * dscale : 0.f);
    }
    *reinterpret_cast<u16x8*>(&dyl[(ry * DYW + xs) * DYC + co0]) = u;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i < HTASK) reinterpret_cast<u16x8*>(h1t)[i] = hv[k];
  }
  if (threadIdx.x < XROWS * IMG / 2) reinterpret_cast<uint32_t*>(xt)[threadIdx.x] = xv;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
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
      for (int mt = 0; mt < 2; ++mt)  // dy2 column xi - kx at tile column xi - kx + 2
        a[mt] = as_bf(*reinterpret_cast<const u16x8*>(&dyl[(arow + mt * 16 + r - kx + 2) * DYC + co0]));  // <= 5 rows past
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bf16x8 bf = tr_frag16(ws, W2S, kc * 32, t * C1 + nt * 16, lane);  // B[k = co][n = ci]
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt][nt] = mfma16(a[mt], bf, acc[mt][nt]);
      }
    }
  }
  // lane: channel ci = nt*16 + r, pixels (yi0 + wave, x = 16mt + 4h + reg)
  float w1acc[2][10];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int t = 0; t < 10; ++t) w1acc[nt][t] = 0.f;
  if (wave < nrows) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int xi = mt * 16 + 4 * h + reg;
        if (xi >= H1) continue;
        float xin[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) xin[t] = bf2f(xt[(wave + t / 3) * IMG + xi + t % 3]);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float dz = bf2f(h1t[(wave * H1 + xi) * C1 + nt * 16 + r]) > 0.f ? acc[mt][nt][reg] : 0.f;
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
    part1[(size_t)blk * P1 + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// ------------------------------------------------------------------- conv2 wgrad partials (MFMA)
constexpr int DYN = C2 + 8;          // dy2 row image [x 32][co]: row stride (elements)
constexpr int HNR = 34;              // h1 rows per ky in the image: x = 0..33 (26..33 zero)
constexpr int HNS = C1 + 8;          // h1 image [ky][x][ci]: row stride (elements)
constexpr int HCHUNKS = 3 * H1 * 4;  // 312 16-byte chunks of h1 per output row (rows y..y+2)
constexpr int WG_BUF = 32 * DYN + 3 * HNR * HNS;  // one stage: dy2 image + h1 image

// Workgroup = a run of consecutive output rows (b, y); per row, K = 24 pixels (padded to 32).  dy2 and
// the three h1 rows it meets are staged row-major exactly as they sit in memory (16-byte writes) and
// both MFMA operands, whose k index is the pixel, are read transposed (tr_frag16); a tap's column
// shift kx is a row offset of the h1 image.  Two LDS stages: the next row's loads are in flight during
// this row's MFMAs and one barrier per row suffices.
constexpr int WG_LDS = 2 * WG_BUF * 2 + 192 * 9 * 4;

__device__ __forceinline__ void conv2_wgrad_block(const u16* __restrict__ dp, const uint8_t* __restrict__ code,
                                                  const u16* __restrict__ h1, float* __restrict__ part2, float dscale, int nrows,
                                                  int rows_per_wg, int blk, char* smem) {
  u16* img = reinterpret_cast<u16*>(smem);
  float (*dbp)[9] = reinterpret_cast<float (*)[9]>(smem + 2 * WG_BUF * 2);
  for (int i = threadIdx.x; i < 2 * WG_BUF; i += 256) img[i] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
  f32x4 acc[18];
#pragma unroll
  for (int n = 0; n < 18; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int row0 = blk * rows_per_wg, row1 = min(nrows, row0 + rows_per_wg);
  // staging tasks: one dy2 (x, 8-channel chunk) if tid < 192; h1 chunks tid and tid + 256
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
    const size_t base = ((size_t)b * H1 + y) * H1 * C1;  // chunk i of rows y..y+2 -> (ky, x, ci0)
    hv0 = *reinterpret_cast<const u16x8*>(h1 + base + (size_t)threadIdx.x * 8);
    if (threadIdx.x + 256 < HCHUNKS) hv1 = *reinterpret_cast<const u16x8*>(h1 + base + (size_t)(threadIdx.x + 256) * 8);
  };
  auto store_h = [&](u16* hn, int i, const u16x8& v) {
    const int ky = i / (H1 * 4), rem = i - ky * (H1 * 4);
    *reinterpret_cast<u16x8*>(&hn[(ky * HNR + (rem >> 2)) * HNS + (rem & 3) * 8]) = v;
  };
  if (row0 < row1) load_row(row0);
  __syncthreads();
  for (int gr = row0, st = 0; gr < row1; ++gr, st ^= 1) {
    u16* dyn = img + st * WG_BUF;
    u16* hn = dyn + 32 * DYN;
    const int y = gr - (gr / H2) * H2;
    if (threadIdx.x < 192) {
      const int q = (y & 1) * 2 + (dx & 1);
      u16x8 u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t c = (uint32_t)(c8 >> (8 * j)) & 0xffu;
        const float v = ((c & 3u) == (uint32_t)q && (c & 12u) == 12u) ? bf2f(d8[j]) * dscale : 0.f;
        db[j] += v;
        u[j] = f2bf(v);
      }
      *reinterpret_cast<u16x8*>(&dyn[dx * DYN + dco0]) = u;
    }
    store_h(hn, threadIdx.x, hv0);
    if (threadIdx.x + 256 < HCHUNKS) store_h(hn, threadIdx.x + 256, hv1);
    __syncthreads();
    if (gr + 1 < row1) load_row(gr + 1);  // in flight during the MFMAs below
    const bf16x8 a = tr_frag16(dyn, DYN, 0, wave * 16, lane);
#pragma unroll
    for (int n = 0; n < 18; ++n) {
      const int t = n >> 1;
      const bf16x8 bf = tr_frag16(hn + (t / 3) * HNR * HNS, HNS, t % 3, (n & 1) * 16, lane);
      acc[n] = mfma16(a, bf, acc[n]);
    }
  }
  float* out = part2 + (size_t)blk * P2;
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

// Both backward GEMMs in one launch (they are independent): blocks [0, n2) compute conv2's weight
// gradient, blocks [n2, n2 + n1) the data gradient + conv1's weight gradient, concurrently.
__global__ __launch_bounds__(256) void conv2_bwd_kernel(const u16* __restrict__ dp, const uint8_t* __restrict__ code,
                                                        const u16* __restrict__ w2, const u16* __restrict__ h1,
                                                        const u16* __restrict__ x, float* __restrict__ part1,
                                                        float* __restrict__ part2, float dscale, int nrows, int rows_per_wg, int n2) {
  __shared__ __attribute__((aligned(16))) char smem[DG_LDS > WG_LDS ? DG_LDS : WG_LDS];
  if ((int)blockIdx.x < n2)
    conv2_wgrad_block(dp, code, h1, part2, dscale, nrows, rows_per_wg, blockIdx.x, smem);
  else
    conv2_dgrad_block(dp, code, w2, h1, x, part1, dscale, blockIdx.x - n2, smem);
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
    for (; k + 28 < n; k += 32) {  // 8 independent loads in flight per round
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(k + 4 * u) * stride];
      s0 += v[0] + v[4];
      s1 += v[1] + v[5];
      s2 += v[2] + v[6];
      s3 += v[3] + v[7];
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

// ------------------------------------------------------------------------ classifier head glue
// fc1 -> ReLU -> dropout -> fc2 -> softmax cross-entropy around two library GEMMs per direction:
// each kernel below replaces 2-5 framework launches (elementwise, bias reduction, fills, casts).
constexpr int HID = 128, NCLS = 10;

// h [B,128] bf16 (fc1 output incl. bias) -> y = keep && h > 0 ? h / (1-p) : 0, code bit0 = keep && h > 0
__global__ __launch_bounds__(256) void relu_dropout_fwd_kernel(const u16* __restrict__ hin, u16* __restrict__ y,
                                                               uint8_t* __restrict__ mask, const float* __restrict__ tptr,
                                                               uint32_t seed, uint32_t drop_thresh, float keep_scale, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t step = (uint32_t)tptr[0];
  const float v = bf2f(hin[i]);
  const bool pass = v > 0.f && (hash3(seed, step, (uint32_t)i) >> 8) >= drop_thresh;
  y[i] = f2bf(pass ? v * keep_scale : 0.f);
  mask[i] = pass ? 1 : 0;
}

// dh = mask ? dy / (1-p) : 0, and fc1's bias gradient = column sums of dh (into the flat buffer).
// Block = 64 columns x 16 row slices.
__global__ __launch_bounds__(1024) void relu_dropout_bwd_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                                u16* __restrict__ dh, u16* __restrict__ gb, float keep_scale,
                                                                int rows, int accumulate) {
  __shared__ float red[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), sl = threadIdx.x >> 6;
  float s = 0.f;
  for (int r = sl; r < rows; r += 16) {
    const size_t i = (size_t)r * HID + c;
    const float v = mask[i] ? bf2f(dy[i]) * keep_scale : 0.f;
    const u16 vb = f2bf(v);
    dh[i] = vb;
    s += bf2f(vb);  // the bias gradient of exactly the dh the weight-gradient GEMM sees
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x & 63];
    if (accumulate) t += bf2f(gb[c]);
    gb[c] = f2bf(t);
  }
}

// Softmax cross-entropy over 10 classes, mean over rows, one block: loss and the unscaled gradient
// dlog = (softmax - onehot) / B in one pass (the backward only scales it).
__global__ __launch_bounds__(256) void xent10_fwd_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                         float* __restrict__ loss, float* __restrict__ dlog, int rows) {
  __shared__ float red[4];
  float s = 0.f;
  const float inv = 1.f / (float)rows;
  for (int r = threadIdx.x; r < rows; r += 256) {
    float z[NCLS], m = -INFINITY;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) {
      z[k] = bf2f(logits[(size_t)r * NCLS + k]);
      m = fmaxf(m, z[k]);
    }
    float e = 0.f;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) {
      z[k] = __expf(z[k] - m);
      e += z[k];
    }
    const int lab = (int)labels[r];
    const float lse = m + __logf(e), ie = 1.f / e;
    s += lse - bf2f(logits[(size_t)r * NCLS + lab]);
#pragma unroll
    for (int k = 0; k < NCLS; ++k) dlog[(size_t)r * NCLS + k] = (z[k] * ie - (k == lab ? 1.f : 0.f)) * inv;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (red[0] + red[1] + red[2] + red[3]) * inv;
}

// dlogits = g * dlog (bf16) and fc2's bias gradient = column sums of it (into the flat buffer).
__global__ __launch_bounds__(256) void xent10_bwd_kernel(const float* __restrict__ dlog, const float* __restrict__ g,
                                                         u16* __restrict__ dlogits, u16* __restrict__ gb, int rows,
                                                         int accumulate) {
  __shared__ float red[25][NCLS];
  const float gs = g[0];
  const int c = threadIdx.x % NCLS, sl = threadIdx.x / NCLS;  // 25 slices x 10 columns (250 threads)
  float s = 0.f;
  if (sl < 25) {
    for (int r = sl; r < rows; r += 25) {
      const u16 vb = f2bf(dlog[(size_t)r * NCLS + c] * gs);
      dlogits[(size_t)r * NCLS + c] = vb;
      s += bf2f(vb);
    }
    red[sl][c] = s;
  }
  __syncthreads();
  if (threadIdx.x < NCLS) {
    float t = 0.f;
    for (int k = 0; k < 25; ++k) t += red[k][threadIdx.x];
    if (accumulate) t += bf2f(gb[threadIdx.x]);
    gb[threadIdx.x] = f2bf(t);
  }
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
  hipLaunchKernelGGL(conv2_bwd_kernel, dim3(n2 + n1), dim3(256), 0, st, bp(dp), code.data_ptr<uint8_t>(), bp(w2), bp(h1), bp(x),
                     part1.data_ptr<float>(), part2.data_ptr<float>(), dscale, nrows, rows_per_wg, n2);
  static_assert(P2 % 64 == 0 && P1 % 64 == 0, "reduce blocks must not straddle the two partial sets");
  hipLaunchKernelGGL(conv_grad_reduce_kernel, dim3((P2 + P1) / 64), dim3(256), 0, st, part1.data_ptr<float>(), n1,
                     part2.data_ptr<float>(), n2, bpm(gw1), bpm(gb1), bpm(gw2), bpm(gb2), accumulate ? 1 : 0);
}

}  // namespace gtk_mnist

namespace gtk_mnist {

std::vector<at::Tensor> relu_dropout_fwd(const at::Tensor& h, const at::Tensor& step, int64_t seed, double p_drop) {
  CHECK_BF16(h);
  TORCH_CHECK(h.dim() == 2 && h.size(1) == HID, "fc1 output must be [B,128]");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kFloat, "step must be a fp32 GPU tensor");
  const int n = (int)h.numel();
  auto y = at::empty_like(h);
  auto mask = at::empty(h.sizes(), h.options().dtype(at::kByte));
  hipLaunchKernelGGL(relu_dropout_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, cur_stream(), bp(h), bpm(y),
                     mask.data_ptr<uint8_t>(), step.data_ptr<float>(), (uint32_t)seed, drop_threshold(p_drop),
                     (float)(1.0 / (1.0 - p_drop)), n);
  return {y, mask};
}

at::Tensor relu_dropout_bwd(const at::Tensor& dy, const at::Tensor& mask, at::Tensor& gb, double p_drop, bool accumulate) {
  CHECK_BF16(dy);
  CHECK_BF16(gb);
  TORCH_CHECK(dy.dim() == 2 && dy.size(1) == HID && mask.numel() == dy.numel() && mask.scalar_type() == at::kByte &&
              mask.is_contiguous() && gb.numel() == HID, "relu_dropout_bwd: shapes");
  auto dh = at::empty_like(dy);
  hipLaunchKernelGGL(relu_dropout_bwd_kernel, dim3(HID / 64), dim3(1024), 0, cur_stream(), bp(dy), mask.data_ptr<uint8_t>(),
                     bpm(dh), bpm(gb), (float)(1.0 / (1.0 - p_drop)), (int)dy.size(0), accumulate ? 1 : 0);
  return dh;
}

std::vector<at::Tensor> xent10_fwd(const at::Tensor& logits, const at::Tensor& labels) {
  CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) == NCLS, "logits must be [B,10]");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
              labels.numel() == logits.size(0), "labels must be int64 [B]");
  const int rows = (int)logits.size(0);
  auto loss = at::empty({}, logits.options().dtype(at::kFloat));
  auto dlog = at::empty({rows, NCLS}, logits.options().dtype(at::kFloat));
  hipLaunchKernelGGL(xent10_fwd_kernel, dim3(1), dim3(256), 0, cur_stream(), bp(logits), labels.data_ptr<int64_t>(),
                     loss.data_ptr<float>(), dlog.data_ptr<float>(), rows);
  return {loss, dlog};
}

at::Tensor xent10_bwd(const at::Tensor& dlog, const at::Tensor& g, at::Tensor& gb, bool accumulate) {
  TORCH_CHECK(dlog.is_cuda() && dlog.scalar_type() == at::kFloat && dlog.is_contiguous() && dlog.dim() == 2 &&
              dlog.size(1) == NCLS, "dlog must be fp32 [B,10]");
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.numel() == 1, "g must be a fp32 GPU scalar");
  CHECK_BF16(gb);
  TORCH_CHECK(gb.numel() == NCLS, "fc2 bias gradient must have 10 entries");
  const int rows = (int)dlog.size(0);
  auto dlogits = at::empty({rows, NCLS}, dlog.options().dtype(at::kBFloat16));
  hipLaunchKernelGGL(xent10_bwd_kernel, dim3(1), dim3(256), 0, cur_stream(), dlog.data_ptr<float>(), g.data_ptr<float>(),
                     bpm(dlogits), bpm(gb), rows, accumulate ? 1 : 0);
  return dlogits;
}

}  // namespace gtk_mnist
