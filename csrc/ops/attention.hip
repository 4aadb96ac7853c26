// Causal GQA flash attention for gfx950 (MFMA 32x32x16 bf16), forward and backward.
//
// Part of the Llama-3 validation workload (BASELINE config 5); replaces the SDPA dispatch (whose
// ROCm flash path is Triton-compiled) with hand-written CDNA4 code.  Head dim 128, bf16 I/O,
// fp32 accumulation and softmax.
//
// Forward (one 256-thread workgroup = 4 waves = 128 queries of one (batch, q-head); KV tiles of 64):
//   * "swapped" QK^T: each wave computes S^T = K . Q^T, so the accumulator holds one QUERY per lane
//     (lane & 31) and 16 keys per 32-key sub-tile in registers; the row max / row sum need only
//     in-lane reductions plus one exchange with lane ^ 32.
//   * that accumulator, rounded to bf16, IS the B operand of O^T += V^T . P^T (§3 "accumulator as the
//     next MFMA's operand"), with V^T fragments gathered by ds_read_b64_tr_b16 from the row-major V
//     tile: no P round trip through LDS.
//   * K and V tiles share one XOR-swizzled LDS image ((b) of guide T10): 16-B chunk ch of row r at
//     256*r + 16*(ch ^ (((r&3)<<2) | ((r>>2)&3))) — conflict-free for both the ds_read_b128 row reads
//     of K and the transposed reads of V.
//   * K/V tiles double-buffered in LDS, the next one staged by LDS-DMA (buffer_load ... lds) under
//     the current tile's softmax and PV, one barrier per tile; query blocks launched heaviest-first,
//     heads XCD-grouped (attn_fwd2_kernel).
//   * output O is written token-major [B, S, H, D] (what the o-projection GEMM consumes) and the
//     row log-sum-exp in log2 units for the backward; optionally O^T from the epilogue.
// Backward (attn_bwd): a pre-kernel (delta = rowsum(dO*O), -lse/c, -delta), then two kernels with no
// cross-workgroup sums:
//   * dK/dV: one workgroup = 128 keys of one (batch, kv-head), sweeping every q-head of the GQA group x
//     32-query slices; key on the lane for S = Q.K^T and dP = dO.V^T, whose P / dS accumulators feed
//     dV^T += dO^T.P and dK^T += Q^T.dS as B operands (dO^T, Q^T by transposed LDS reads); a 3-slot
//     LDS-DMA slice ring, the dV/dK products of slice i under the softmax of slice i+1.
//   * dQ: forward-shaped (query on the lane), dQ^T += K^T.dS^T accumulated in registers.
// Earlier generations (forward v1 with one LDS buffer, backward v1 with fp32 dQ atomics, backward v2
// with synchronous slice staging) were measured, retired, and live in git history before round 2.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cmath>
#include <cstdint>

namespace gtk_attn {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 128;
constexpr int BQ = 128;  // forward: queries per workgroup
constexpr int BK = 64;   // forward: keys per tile
constexpr int KB = 128;  // backward: keys per workgroup
constexpr int QT = 32;   // backward: queries per slice

#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

// byte offset of 16-B chunk `ch` of row `row` in a [rows][128 x bf16] swizzled image
__device__ __forceinline__ int swz(int row, int ch) { return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }
// accumulator register -> row of a 32x32 MFMA tile (lane half hh)
__device__ __forceinline__ int crow(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int off) { return *reinterpret_cast<const bf16x8*>(base + off); }

__device__ __forceinline__ s16x4 lds_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(base + off));
}

// Two transposed 4-element reads -> one bf16x8 MFMA operand.  Whole-vector bit casts only: on ROCm
// 7.2 (clang 22) a per-element __builtin_bit_cast(__bf16, v[j]) of the tr-read result is folded to
// element 0 for every j (one ds_read_b64_tr_b16 + v_perm broadcast in the .s), silently wrong.
__device__ __forceinline__ bf16x8 cat8(s16x4 lo, s16x4 hi) {
  return __builtin_shufflevector(__builtin_bit_cast(bf16x4, lo), __builtin_bit_cast(bf16x4, hi), 0, 1, 2, 3, 4, 5, 6, 7);
}

// Transposed A fragment of a 32x32x16 MFMA whose k index walks ROWS of a [rows][128] swizzled image
// and whose output row walks COLUMNS: element j of lane (r, hh) = img[row_of(j)][col0 + r] where
// rows are r_lo + {0..3} (j < 4) and r_hi + {0..3} (j >= 4).  r_lo/r_hi are per-half (caller adds 4*hh).
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int lane, int r_lo, int r_hi, int col0) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = col0 + 16 * (g & 1);  // first column this 16-lane group delivers
  const int ch = (col >> 3) + (p >> 1);
  s16x4 lo = lds_tr(img, swz(r_lo + q, ch) + 8 * (p & 1));
  s16x4 hi = lds_tr(img, swz(r_hi + q, ch) + 8 * (p & 1));
  return cat8(lo, hi);
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int base) {
  bf16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (__bf16)acc[base + j];
  return out;
}

__device__ __forceinline__ bf16x8 pack8a(const float* x, int base) {
  bf16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (__bf16)x[base + j];
  return out;
}

// Empty asm statements that "modify" their operands: code computing those values cannot move across
// them, and volatile asm keeps its order with the other volatile asm (the dV/dK MFMAs of dK/dV v7), so a
// pair of pins fixes which MFMA gap a piece of VALU issues in.  No instruction is emitted.
__device__ __forceinline__ void pin2(float& a, float& b) { asm volatile("" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ void pin4(float& a, float& b, float& c, float& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void pin16(float* x) {
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
  asm volatile("" : "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]));
}
__device__ __forceinline__ void pin_b(bf16x8& a, bf16x8& b) { asm volatile("" : "+v"(a), "+v"(b)); }
__device__ __forceinline__ void pin_b1(bf16x8& a) { asm volatile("" : "+v"(a)); }

// raw v_exp_f32 (2^x): no denormal range reduction — softmax terms below 2^-126 are 0 either way
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 16-byte LDS-DMA: lane i's 16 bytes from g land at lds_base + 16 i (lds_base wave-uniform, -> M0)
__device__ __forceinline__ void glds16(const u16* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g, (LDS_AS void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ==================================================================================== forward

// XCD-aware (batch*head) order: workgroups are dealt round-robin over the 8 XCDs (id % 8), so map
// consecutive ids of one XCD to consecutive heads — the q-heads of a GQA group (which read the same
// K/V) then run on one XCD and share its L2.  Identity when the head count is not a multiple of 8.
__device__ __forceinline__ int xcd_head(int id, int n) { return (n & 7) ? id : (id & 7) * (n >> 3) + (id >> 3); }

// LDS-DMA staging of one [BK=64][128] K tile and V tile into the swizzled images (K at img, V at
// img + 16 KiB) by a 4-wave workgroup: wave w fills rows 16w .. 16w+15 with 4 + 4
// buffer_load_dwordx4 ... lds (1 KiB = 4 rows each).  The destination is lane-linear, so the XOR
// swizzle goes on the SOURCE offset: lane (row R, slot p) fetches chunk p ^ f(R), which makes
// swz(R, chunk) == 256 R + 16 p.  Descriptors are built from wave-uniform values only (no
// waterfall loops); the per-tile step is one scalar offset.
struct KVStage {
  __amdgpu_buffer_rsrc_t krs, vrs;
  uint32_t voff[4];
  int w;
  __device__ __forceinline__ KVStage(const u16* kbase, const u16* vbase, int S, int w_, int lane) : w(w_) {
    const uint32_t bytes = (uint32_t)((size_t)S * D * 2);
    krs = __builtin_amdgcn_make_buffer_rsrc((void*)kbase, 0, bytes, 0x00020000);
    vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vbase, 0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int R = 16 * w + 4 * i + (lane >> 4);
      voff[i] = (uint32_t)(R * D * 2 + 16 * ((lane & 15) ^ (((R & 3) << 2) | ((R >> 2) & 3))));
    }
  }
  __device__ __forceinline__ void load(int kt, char* img) const {
    const uint32_t soff = (uint32_t)kt * (BK * D * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (LDS_AS void*)(img + (16 * w + 4 * i) * 256), 16, voff[i], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (LDS_AS void*)(img + BK * D * 2 + (16 * w + 4 * i) * 256), 16, voff[i], soff,
                                               0, 0);
    }
  }
};

// Every wave's outstanding LDS-DMA has landed AND every LDS read it issued has returned, then a
// barrier: after it, the tile just staged is visible to the workgroup and the tile just read may be
// overwritten by the next DMA.  Both halves of that contract are spelled out here rather than left to
// the barrier's fence lowering or to the compiler's LDS-DMA alias analysis.
__device__ __forceinline__ void dma_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// Forward v2: same math as attn_fwd_kernel, restructured for the CDNA4 pipes.
//   * grid (B*H, S/128): x = head fastest, so dispatch order is heaviest query block first across
//     ALL heads (LPT order for the causal triangle), heads XCD-grouped (xcd_head).
//   * K/V double-buffered in LDS (2 x 32 KiB), ONE barrier per tile.  The next tile arrives by
//     LDS-DMA (buffer_load ... lds through a wave-uniform descriptor, swizzle on the source offset)
//     into the other buffer, issued after QK^T and retired before the barrier: no staging
//     registers, no ds_write pass, per-tile addressing in one scalar.
//   * K fragments read 8 ahead of the QK^T chain (sched_group_barrier), not one pair at a time.
//   * scale folded into the exponent: p = 2^(s*c - m) with one v_fma + v_exp per score; the max is
//     taken on raw scores (c > 0) with v_max3.  Only the last two tiles of a block can need the
//     causal mask or be invisible to a wave: the main loop is branch-free, those two are peeled.
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));  // no IEEE canonicalising v_max per operand
  return r;
}

// Running-max slack (log2 units, guide T13): the max used for the exponent is only raised when a
// row's max exceeds it by more than kMaxSlack, so P <= 2^kMaxSlack (exact after the final 1/l) and
// the O rescale, 64 multiplies per wave, runs on a few early tiles instead of on most tiles.
constexpr float kMaxSlack = 8.f;

__device__ __forceinline__ float xhalf_max(float x) {  // max(x[lane], x[lane ^ 32])
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

__global__ __launch_bounds__(256, 2) void attn_fwd2_kernel(const u16* __restrict__ q, const u16* __restrict__ k,
                                                           const u16* __restrict__ v, u16* __restrict__ o,
                                                           float* __restrict__ lse2, int H, int Hkv, int S, float c,
                                                           u16* __restrict__ ot = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BK * D * 2];  // [buf][K image | V image]
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nqb = gridDim.y;
  const int qb = nqb - 1 - blockIdx.y;  // heaviest first
  const int bh = xcd_head(blockIdx.x, gridDim.x), b = bh / H, hq = bh % H, hk = hq / (H / Hkv);
  const u16* qp = q + ((size_t)(b * H + hq) * S) * D;
  const size_t kvoff = ((size_t)(b * Hkv + hk) * S) * D;
  const int q0 = qb * BQ + w * 32;
  const int myq = q0 + r;

  bf16x8 qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + (size_t)myq * D + 16 * s + 8 * hh);

  f32x16 oacc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) oacc[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;  // m in units of log2 (score * c)

  const int ntiles = (qb * BQ + BQ) / BK;
  const KVStage stage(k + kvoff, v + kvoff, S, w, lane);
  auto gload = [&](int kt, char* img) { stage.load(kt, img); };

  // one KV tile: QK^T, DMA of the next tile, online softmax, PV.  `masked` (compile-time at each
  // call) adds the causal mask for the wave's diagonal tiles.
  auto tile = [&](int kt, bool masked) {
    char* kimg = smem + (kt & 1) * (2 * BK * D * 2);
    char* vimg = kimg + BK * D * 2;
    const int key0 = kt * BK;
    f32x16 s0 = f32x16{}, s1 = f32x16{};
    __builtin_amdgcn_s_setprio(1);  // MFMA phases outrank the other wave's softmax VALU (ping-pong)
    {
      bf16x8 kf0[8], kf1[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        kf0[s] = lds_b128(kimg, swz(r, 2 * s + hh));
        kf1[s] = lds_b128(kimg, swz(32 + r, 2 * s + hh));
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        s0 = mfma(kf0[s], qf[s], s0);
        s1 = mfma(kf1[s], qf[s], s1);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // 8 reads ahead, then read/MFMA pairs
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x8, 8, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < ntiles) gload(kt + 1, smem + ((kt + 1) & 1) * (2 * BK * D * 2));  // lands under softmax + PV
    if (masked) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k0i = key0 + crow(i, hh);
        if (k0i > myq) s0[i] = -INFINITY;
        if (k0i + 32 > myq) s1[i] = -INFINITY;
      }
    }
    float mx = max3(s0[0], s1[0], s0[1]);
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = max3(mx, s1[i], i + 1 < 16 ? s0[i + 1] : s1[i]);
    const float mrow = xhalf_max(mx) * c;
    // per row (a row's frame must depend on its own visible scores only: causality is bitwise);
    // the wave-uniform `resc` only gates the rescale branch, alpha == 1 exactly on unmoved rows
    const float mnew = mrow > m + kMaxSlack ? mrow : m;
    const bool resc = __any(mnew != m);
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s0[i] = fexp2(fmaf(s0[i], c, -mnew));
      s1[i] = fexp2(fmaf(s1[i], c, -mnew));
      rs += s0[i] + s1[i];
    }
    rs += __shfl_xor(rs, 32, 64);
    if (resc) {  // alpha == 1 everywhere otherwise
      const float alpha = fexp2(m - mnew);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    }
    l += rs;
    m = mnew;
    const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 8), p10 = pack8(s1, 0), p11 = pack8(s1, 8);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col0 = 32 * dt;
      oacc[dt] = mfma(tr_frag(vimg, lane, 0 + 4 * hh, 8 + 4 * hh, col0), p00, oacc[dt]);
      oacc[dt] = mfma(tr_frag(vimg, lane, 16 + 4 * hh, 24 + 4 * hh, col0), p01, oacc[dt]);
      oacc[dt] = mfma(tr_frag(vimg, lane, 32 + 4 * hh, 40 + 4 * hh, col0), p10, oacc[dt]);
      oacc[dt] = mfma(tr_frag(vimg, lane, 48 + 4 * hh, 56 + 4 * hh, col0), p11, oacc[dt]);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  gload(0, smem);
  dma_sync();
  // tiles 0 .. ntiles-3 lie entirely below every query of the block: no mask, no visibility test
  int kt = 0;
  for (; kt < ntiles - 2; ++kt) {
    tile(kt, false);
    dma_sync();
  }
  // the block's diagonal: tile ntiles-2 covers keys [128 qb, 128 qb + 64), ntiles-1 the next 64
  for (; kt < ntiles; ++kt) {
    const int key0 = kt * BK;
    if (key0 <= q0 + 31) {
      tile(kt, key0 + BK - 1 > q0);
    } else if (kt + 1 < ntiles) {
      gload(kt + 1, smem + ((kt + 1) & 1) * (2 * BK * D * 2));
    }
    dma_sync();
  }
  const float inv = 1.f / l;
  u16* orow = o + (((size_t)b * S + myq) * (size_t)(H) + hq) * D;
  // O^T [H*D, B*S] (ot != nullptr): the o-projection's x^T for its NT-layout weight gradient, written
  // from an LDS image of the block's [128 d][128 q] tile (the loop's last dma_sync retired every LDS
  // read, so the K/V ring is free) as 256-B row segments, instead of by a transpose pass in the
  // backward.  Same bf16 values as O.  Row stride 136 elements (272 B) staggers the banks.
  constexpr int kOtStride = 136;
  u16* otl = reinterpret_cast<u16*>(smem);
  // T21: lane half hh holds columns 8k + 4hh .. +3 of its row; one v_permlane32_swap per dword of a
  // pair of column groups (k, k+1) gives every lane 16 contiguous bytes (lanes 0-31: group k, lanes
  // 32-63: group k+1): 8 dwordx4 stores per lane instead of 16 dwordx2
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; g4 += 2) {
      u16x4 va, vb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        va[e] = f2bf(oacc[dt][4 * g4 + e] * inv);
        vb[e] = f2bf(oacc[dt][4 * g4 + 4 + e] * inv);
      }
      if (ot) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          otl[(32 * dt + 8 * g4 + 4 * hh + e) * kOtStride + w * 32 + r] = va[e];
          otl[(32 * dt + 8 * g4 + 8 + 4 * hh + e) * kOtStride + w * 32 + r] = vb[e];
        }
      }
      const auto a = __builtin_bit_cast(uint2, va), bb = __builtin_bit_cast(uint2, vb);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a.x, bb.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a.y, bb.y, false, false);
      const uint4 out = {s0[0], s1[0], s0[1], s1[1]};
      *reinterpret_cast<uint4*>(orow + 32 * dt + 8 * g4 + 8 * hh) = out;
    }
  if (hh == 0) lse2[(size_t)(b * H + hq) * S + myq] = m + log2f(l);
  if (ot) {
    __syncthreads();
    const int d = t >> 1, half = t & 1;
    const size_t BS = (size_t)(gridDim.x / H) * S;
    u16* dst = ot + ((size_t)hq * D + d) * BS + (size_t)b * S + (size_t)qb * BQ + 64 * half;
    const u16* srcl = otl + d * kOtStride + 64 * half;
#pragma unroll
    for (int j = 0; j < 8; ++j) reinterpret_cast<u16x8*>(dst)[j] = reinterpret_cast<const u16x8*>(srcl)[j];
  }
}

// ==================================================================================== backward
// delta[b, h, q] = sum_d dO[b, q, h, d] * O[b, q, h, d] (one 16-lane group per row; dQ reads it), plus
// what dK/dV starts its S / dP chains from: nls = -lse2 / c, ndl = -delta
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                            const float* __restrict__ lse2, float* __restrict__ delta,
                                                            float* __restrict__ nls, float* __restrict__ ndl, int B, int H,
                                                            int S, float inv_c) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);  // row = (b*S + s)*H + h
  const int i = threadIdx.x & 15;
  if (row >= B * S * H) return;
  const u16x8 a = reinterpret_cast<const u16x8*>(dout + (size_t)row * D)[i];
  const u16x8 bb = reinterpret_cast<const u16x8*>(out + (size_t)row * D)[i];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += bf2f(a[j]) * bf2f(bb[j]);
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off, 16);
  if (i == 0) {
    const int h = row % H, bs = row / H, sidx = bs % S, bidx = bs / S;
    const size_t o = ((size_t)bidx * H + h) * S + sidx;
    delta[o] = s;
    ndl[o] = -s;
    nls[o] = -lse2[o] * inv_c;
  }
}

// ============================================================================ backward dK/dV
// The split dK/dV decomposition: one workgroup = 128 keys of one (batch, kv-head), sweeping every q-head
// of the GQA group x 32-query slices, key on the lane; each lane's K and V rows live in registers for
// the whole kernel.  Q, dO, -lse/c and -delta of a slice arrive by LDS-DMA into a 3-slot ring, one slice
// ahead, with one barrier per slice.  Each slice's dV^T += dO^T.P and dK^T += Q^T.dS products are
// deferred by one slice, so its softmax / dS VALU runs under the previous slice's products.  Only the
// first KB/QT slices of each q-head touch the block's diagonal: mask code runs there only.
//
// Round 5 (v7) re-budgeted the registers of the round-4 kernel (v5).  v5 held ~460 registers at one
// wave per SIMD; past 256 the compiler selects the AGPR form for EVERY MFMA, so S / dP landed in AGPRs
// and each slice paid ~100 v_accvgpr_read / write / mov to bring them to the softmax VALU and back.
// Now (hipcc -S: 252 VGPRs + 128 AGPRs, no accumulator moves in the loop):
//   * -lse/c and -delta enter as the S and dP chains' initial accumulators (the pre-kernel writes them
//     negated and pre-divided): p = 2^(c S') and dS = p dP' need no lse / delta registers, no subtract;
//   * the long-lived dV^T / dK^T accumulators (128 registers) are pinned in AGPRs by their MFMAs' asm
//     constraints, and the S / dP MFMAs take the VGPR form (attention.hip is built with
//     -amdgpu-mfma-vgpr-form); each gap's softmax VALU is pinned between two of those asm MFMAs by
//     empty asm statements on its operands;
//   * the transposed dO^T / Q^T fragments are read two products ahead of their use (12 registers
//     instead of 64), which leaves room to read this slice's rows and init quads ahead of the S / dP
//     chains;
//   * the next slice's DMA is issued at the step start, into a slot passed as a __restrict__ pointer
//     (so no read of this step waits for it): a whole step to land.
// Measured at B 4 x 4096 (profiles/r05_attn7): 1434 -> 1009 us per dK/dV launch, MFMA busy 39 -> 52 %,
// whole backward -14.6 %.  v3 / v4 / v5 and the v7 A/B variants are retired; their records are
// profiles/r04_attn, r04_maskbr, r04_split, r04_vpg, r05_attn7.
constexpr int SL_Q = 0, SL_DO = QT * D * 2, SL_LSE = 2 * QT * D * 2, SL_DEL = SL_LSE + 256, SL_BYTES = SL_DEL + 256;

__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv_kernel(const u16* __restrict__ q, const u16* __restrict__ k,
                                                                const u16* __restrict__ v, const u16* __restrict__ dout,
                                                                const float* __restrict__ nls, const float* __restrict__ ndl,
                                                                u16* __restrict__ dk, u16* __restrict__ dv, int H, int Hkv,
                                                                int S, float c, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[3 * SL_BYTES];  // slice ring
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int kb = blockIdx.y;
  const int bk = xcd_head(blockIdx.x, gridDim.x), b = bk / Hkv, hk = bk % Hkv, G = H / Hkv;
  const size_t kvoff = ((size_t)(b * Hkv + hk) * S + (size_t)kb * KB) * D;
  const int krow = w * 32 + r, mykey = kb * KB + krow, kmin = kb * KB + w * 32;
  bf16x8 kf[8], vf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(k + kvoff + (size_t)krow * D + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(v + kvoff + (size_t)krow * D + 16 * s + 8 * hh);
  }
  f32x16 dvt[4], dkt[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dvt[dt] = dkt[dt] = f32x16{};
  // the zeroing writes settle before the first asm MFMA reads them as its accumulator
  asm volatile("s_nop 1" : "+a"(dvt[0]), "+a"(dvt[1]), "+a"(dvt[2]), "+a"(dvt[3]), "+a"(dkt[0]), "+a"(dkt[1]), "+a"(dkt[2]),
                 "+a"(dkt[3]));
  const int qt0 = (kb * KB) / QT, nqt = S / QT - qt0, nslice = G * nqt;

  const uint32_t qbytes = (uint32_t)((size_t)H * S * D * 2), dbytes = (uint32_t)((size_t)S * H * D * 2);
  const auto qrs = __builtin_amdgcn_make_buffer_rsrc((void*)(q + (size_t)b * H * S * D), 0, qbytes, 0x00020000);
  const auto drs = __builtin_amdgcn_make_buffer_rsrc((void*)(dout + (size_t)b * S * H * D), 0, dbytes, 0x00020000);
  const auto lrs = __builtin_amdgcn_make_buffer_rsrc((void*)((w == 0 ? nls : ndl) + (size_t)b * H * S), 0,
                                                     (uint32_t)((size_t)H * S * 4), 0x00020000);
  uint32_t qv[2], dvo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = 8 * w + 4 * i + (lane >> 4);
    const uint32_t ch16 = 16 * ((lane & 15) ^ (((R & 3) << 2) | ((R >> 2) & 3)));
    qv[i] = (uint32_t)(R * D * 2) + ch16;
    dvo[i] = (uint32_t)(R * H * D * 2) + ch16;
  }
  // slices are walked in (q-head, query tile) order; (sh, sj) of a slice are stepped, not divided out
  auto sload = [&](int sh, int sj, char* buf) {
    const int hq = hk * G + sh, qbase = (qt0 + sj) * QT;
    const uint32_t qs = (uint32_t)(((size_t)hq * S + qbase) * D * 2), ds = (uint32_t)(((size_t)qbase * H + hq) * D * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (LDS_AS void*)(buf + SL_Q + (8 * w + 4 * i) * 256), 16, qv[i], qs, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, (LDS_AS void*)(buf + SL_DO + (8 * w + 4 * i) * 256), 16, dvo[i], ds, 0, 0);
    }
    if (w < 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, (LDS_AS void*)(buf + (w == 0 ? SL_LSE : SL_DEL)), 4, 4 * lane,
                                               (uint32_t)(((size_t)hq * S + qbase) * 4), 0, 0);
  };
  int cur_h = 0, cur_j = 0;  // this step's slice
  // dV^T / dK^T += A . B, the accumulator pinned to AGPRs by the asm constraint
  auto acc_mfma = [&](f32x16& acc, bf16x8 a, bf16x8 bb) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(bb));
  };
  struct Packs {
    bf16x8 p0, p1, d0, d1;
  };

  Packs prev{};
  {  // the first step's deferred products read ring(2): zeros, not stale LDS bits
    u16x8* z = reinterpret_cast<u16x8*>(smem + 2 * SL_BYTES);
    for (int i = t; i < SL_BYTES / 16; i += 256) z[i] = u16x8{};
  }
  __syncthreads();
  sload(0, 0, smem);
  dma_sync();
  // buf: this slice; pbuf: the previous one (its deferred dV/dK products); nbuf: the slot the next
  // slice's DMA fills.  As __restrict__ parameters the three are provably disjoint, so no read of buf /
  // pbuf waits for the DMA into nbuf, issued first: it has a whole step to land
  auto step = [&](int idx, const char* __restrict__ buf, const char* __restrict__ pbuf, char* __restrict__ nbuf) {
    const int nj = cur_j + 1 == nqt ? 0 : cur_j + 1, nh = cur_j + 1 == nqt ? cur_h + 1 : cur_h;
    if (idx + 1 < nslice) sload(nh, nj, nbuf);
    // (1) this slice's -lse/c, -delta (the S / dP chains' initial accumulators) and its rows
    f32x16 sacc, dpacc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(buf + SL_LSE + 4 * (8 * g + 4 * hh));
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(buf + SL_DEL + 4 * (8 * g + 4 * hh));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sacc[4 * g + e] = l4[e];
        dpacc[4 * g + e] = d4[e];
      }
    }
    bf16x8 qa[8], da[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      qa[s] = lds_b128(buf + SL_Q, swz(r, 2 * s + hh));
      da[s] = lds_b128(buf + SL_DO, swz(r, 2 * s + hh));
    }
    // the previous slice's transposed dO^T / Q^T fragment ti (A operand of dV^T / dK^T product ti)
    auto tfrag = [&](int ti) {
      const int dt = ti >> 2, part = ti & 3;
      return tr_frag(pbuf + (part < 2 ? SL_DO : SL_Q), lane, (part & 1) * 16 + 4 * hh, (part & 1) * 16 + 8 + 4 * hh, 32 * dt);
    };
    // dV/dK product i in issue order: accumulators round-robin, so an accumulator's two products are
    // 4 MFMAs apart
    auto tix = [](int i) { return 4 * (i & 3) + (i >> 2); };
    // (2) S' = S - lse/c and dP' = dP - delta.  The transposed fragments of phase (3) are read two
    // products ahead of their use; the first two here.  16 of the step's 28 LDS reads (8 init quads, 16
    // rows, 4 transposed halves) go before the first MFMA, then one per MFMA: every MFMA's rows were
    // issued ~7 MFMAs earlier (fewer up front and the compiler streams the rows through one register
    // quad, each MFMA waiting on its own read)
    bf16x8 ta[16];
    ta[tix(0)] = tfrag(tix(0));
    ta[tix(1)] = tfrag(tix(1));
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      sacc = mfma(qa[s], kf[s], sacc);
      dpacc = mfma(da[s], vf[s], dpacc);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
    for (int g = 0; g < 12; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    // (3) softmax / dS of this slice under the deferred dV/dK MFMAs of the previous one
    // diagonal slices (the block's first KB/QT query tiles) mask from qbase; slices wholly above this
    // wave's keys are dead (every score masked)
    const int qbase = (qt0 + cur_j) * QT;
    const bool dead = cur_j < KB / QT && qbase + QT - 1 < kmin;
    const int kill_from = dead ? -(1 << 30) : (cur_j < KB / QT ? qbase : 1 << 30);
    Packs cur;
    // The dV/dK MFMAs are asm statements, which the scheduling-group barriers do not see; each gap's
    // VALU is pinned between its two MFMAs instead: an empty asm right after MFMA i "writes" the gap's
    // inputs and another right before MFMA i+1 "reads" its outputs (no instructions emitted).  LDS reads
    // keep their source position relative to the (side-effecting) asm statements.
    float sp[16], dp[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) sp[i] = sacc[i], dp[i] = dpacc[i];
    auto M = [&](int i) {
      const int ti = tix(i), dt = ti >> 2, part = ti & 3;
      f32x16& acc = part < 2 ? dvt[dt] : dkt[dt];
      const bf16x8 bb = part == 0 ? prev.p0 : part == 1 ? prev.p1 : part == 2 ? prev.d0 : prev.d1;
      acc_mfma(acc, ta[ti], bb);
      if (i + 2 < 16) ta[tix(i + 2)] = tfrag(tix(i + 2));
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // gaps 0-7: p = 2^(c S') for two scores each (mul + exp: 24 cycles)
      M(i);
      pin2(sp[2 * i], sp[2 * i + 1]);
      sp[2 * i] = fexp2(sp[2 * i] * c);
      sp[2 * i + 1] = fexp2(sp[2 * i + 1] * c);
      pin2(sp[2 * i], sp[2 * i + 1]);
    }
    M(8);  // gap 8: the causal mask (diagonal / dead slices only), P's two packs
    pin16(sp);
    if (kill_from != (1 << 30)) {  // wave-uniform
#pragma unroll
      for (int i = 0; i < 16; ++i) sp[i] = (mykey - crow(i, hh) > kill_from) ? 0.f : sp[i];
    }
    cur.p0 = pack8a(sp, 0);
    cur.p1 = pack8a(sp, 8);
    pin_b(cur.p0, cur.p1);
#pragma unroll
    for (int i = 9; i < 13; ++i) {  // gaps 9-12: dS = p dP' for four scores each
      M(i);
      const int o = 4 * (i - 9);
      pin4(dp[o], dp[o + 1], dp[o + 2], dp[o + 3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) dp[o + e] *= sp[o + e];
      pin4(dp[o], dp[o + 1], dp[o + 2], dp[o + 3]);
    }
    M(13);  // gaps 13-14: dS's packs
    pin4(dp[0], dp[1], dp[2], dp[3]);
    pin4(dp[4], dp[5], dp[6], dp[7]);
    cur.d0 = pack8a(dp, 0);
    pin_b1(cur.d0);
    M(14);
    pin4(dp[8], dp[9], dp[10], dp[11]);
    pin4(dp[12], dp[13], dp[14], dp[15]);
    cur.d1 = pack8a(dp, 8);
    pin_b1(cur.d1);
    M(15);
    __builtin_amdgcn_sched_barrier(0);
    prev = cur;
    cur_h = nh, cur_j = nj;
    dma_sync();
  };
  int idx = 0;
  char* const s0 = smem;
  char* const s1 = smem + SL_BYTES;
  char* const s2 = smem + 2 * SL_BYTES;
  for (; idx + 3 <= nslice; idx += 3) {
    step(idx, s0, s2, s1);
    step(idx + 1, s1, s0, s2);
    step(idx + 2, s2, s1, s0);
  }
  if (idx < nslice) step(idx, s0, s2, s1);
  if (idx + 1 < nslice) step(idx + 1, s1, s0, s2);
  {  // the last slice's deferred dV/dK products
    const char* pbuf = smem + ((nslice - 1) % 3) * SL_BYTES;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      acc_mfma(dvt[dt], tr_frag(pbuf + SL_DO, lane, 0 + 4 * hh, 8 + 4 * hh, 32 * dt), prev.p0);
      acc_mfma(dvt[dt], tr_frag(pbuf + SL_DO, lane, 16 + 4 * hh, 24 + 4 * hh, 32 * dt), prev.p1);
      acc_mfma(dkt[dt], tr_frag(pbuf + SL_Q, lane, 0 + 4 * hh, 8 + 4 * hh, 32 * dt), prev.d0);
      acc_mfma(dkt[dt], tr_frag(pbuf + SL_Q, lane, 16 + 4 * hh, 24 + 4 * hh, 32 * dt), prev.d1);
    }
  }
  // asm MFMAs are invisible to the hazard recognizer: their results settle before the reads
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(dvt[0]), "+a"(dvt[1]), "+a"(dvt[2]), "+a"(dvt[3]), "+a"(dkt[0]),
                 "+a"(dkt[1]), "+a"(dkt[2]), "+a"(dkt[3]));
  u16* dkrow = dk + ((size_t)(b * Hkv + hk) * S + mykey) * D;
  u16* dvrow = dv + ((size_t)(b * Hkv + hk) * S + mykey) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u16x4 a4, b4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a4[e] = f2bf(dkt[dt][4 * g4 + e] * scale);
        b4[e] = f2bf(dvt[dt][4 * g4 + e]);
      }
      *reinterpret_cast<u16x4*>(dkrow + 32 * dt + 8 * g4 + 4 * hh) = a4;
      *reinterpret_cast<u16x4*>(dvrow + 32 * dt + 8 * g4 + 4 * hh) = b4;
    }
}

// dQ: forward-shaped (query on the lane), dQ^T += K^T.dS^T accumulated in registers; LDS-DMA
// double-buffered K/V tiles with one barrier per tile, the block's diagonal tiles peeled out of a
// branch-free main loop, LPT + XCD-grouped grid (B*H, S/128).  The tile's LDS images are __restrict__
// parameters of an inlined function, so the compiler's LDS-DMA wait tracking sees the reads and the
// next tile's DMA as disjoint and puts no mid-tile wait in front of the first transposed K read (the
// round-3 dq2 did; 1.2 % slower whole backward at B 4, profiles/r04_attn).  The ordering the double
// buffer needs is dma_sync()'s explicit vmcnt(0) lgkmcnt(0) + barrier at the end of every tile.
template <bool kMasked>
__device__ __forceinline__ void dq_tile_na(const char* __restrict__ kimg, const char* __restrict__ vimg,
                                           char* __restrict__ nimg, bool prefetch, const KVStage& stage, int kt,
                                           const bf16x8 (&qf)[8], const bf16x8 (&df)[8], f32x16 (&dqt)[4], float lse_q,
                                           float del_q, int lane, int r, int hh, int myq, float c) {
  const int key0 = kt * BK;
  f32x16 s0 = f32x16{}, s1 = f32x16{}, e0 = f32x16{}, e1 = f32x16{};
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const bf16x8 k0 = lds_b128(kimg, swz(r, 2 * s + hh)), k1 = lds_b128(kimg, swz(32 + r, 2 * s + hh));
    const bf16x8 v0 = lds_b128(vimg, swz(r, 2 * s + hh)), v1 = lds_b128(vimg, swz(32 + r, 2 * s + hh));
    s0 = mfma(k0, qf[s], s0);
    s1 = mfma(k1, qf[s], s1);
    e0 = mfma(v0, df[s], e0);
    e1 = mfma(v1, df[s], e1);
  }
  __builtin_amdgcn_s_setprio(0);
  if (prefetch) stage.load(kt + 1, nimg);  // lands under the dQ MFMAs
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float p0 = fexp2(fmaf(s0[i], c, -lse_q));
    float p1 = fexp2(fmaf(s1[i], c, -lse_q));
    if (kMasked) {
      const int kk = key0 + crow(i, hh);
      if (kk > myq) p0 = 0.f;
      if (kk + 32 > myq) p1 = 0.f;
    }
    s0[i] = p0 * (e0[i] - del_q);
    s1[i] = p1 * (e1[i] - del_q);
  }
  const bf16x8 d00 = pack8(s0, 0), d01 = pack8(s0, 8), d10 = pack8(s1, 0), d11 = pack8(s1, 8);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    dqt[dt] = mfma(tr_frag(kimg, lane, 0 + 4 * hh, 8 + 4 * hh, 32 * dt), d00, dqt[dt]);
    dqt[dt] = mfma(tr_frag(kimg, lane, 16 + 4 * hh, 24 + 4 * hh, 32 * dt), d01, dqt[dt]);
    dqt[dt] = mfma(tr_frag(kimg, lane, 32 + 4 * hh, 40 + 4 * hh, 32 * dt), d10, dqt[dt]);
    dqt[dt] = mfma(tr_frag(kimg, lane, 48 + 4 * hh, 56 + 4 * hh, 32 * dt), d11, dqt[dt]);
  }
  __builtin_amdgcn_s_setprio(0);
}

__global__ __launch_bounds__(256, 2) void attn_bwd_dq2n_kernel(const u16* __restrict__ q, const u16* __restrict__ k,
                                                               const u16* __restrict__ v, const u16* __restrict__ dout,
                                                               const float* __restrict__ lse2, const float* __restrict__ delta,
                                                               u16* __restrict__ dq, int H, int Hkv, int S, float c, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BK * D * 2];  // [buf][K image | V image]
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nqb = gridDim.y, qb = nqb - 1 - blockIdx.y;
  const int bh = xcd_head(blockIdx.x, gridDim.x), b = bh / H, hq = bh % H, hk = hq / (H / Hkv);
  const size_t kvoff = ((size_t)(b * Hkv + hk) * S) * D;
  const int q0 = qb * BQ + w * 32, myq = q0 + r;
  const u16* qrow = q + ((size_t)(b * H + hq) * S + myq) * D;
  const u16* dorow = dout + (((size_t)b * S + myq) * H + hq) * D;
  bf16x8 qf[8], df[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s + 8 * hh);
    df[s] = *reinterpret_cast<const bf16x8*>(dorow + 16 * s + 8 * hh);
  }
  const float lse_q = lse2[(size_t)(b * H + hq) * S + myq], del_q = delta[(size_t)(b * H + hq) * S + myq];
  f32x16 dqt[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dqt[dt] = f32x16{};
  const int ntiles = (qb * BQ + BQ) / BK;
  const KVStage stage(k + kvoff, v + kvoff, S, w, lane);
  auto tile = [&](int kt, bool masked) {
    const char* kimg = smem + (kt & 1) * (2 * BK * D * 2);
    char* nimg = smem + ((kt + 1) & 1) * (2 * BK * D * 2);
    if (masked)
      dq_tile_na<true>(kimg, kimg + BK * D * 2, nimg, kt + 1 < ntiles, stage, kt, qf, df, dqt, lse_q, del_q, lane, r, hh, myq, c);
    else
      dq_tile_na<false>(kimg, kimg + BK * D * 2, nimg, kt + 1 < ntiles, stage, kt, qf, df, dqt, lse_q, del_q, lane, r, hh, myq, c);
  };
  stage.load(0, smem);
  dma_sync();
  int kt = 0;
  for (; kt < ntiles - 2; ++kt) {
    tile(kt, false);
    dma_sync();
  }
  for (; kt < ntiles; ++kt) {
    const int key0 = kt * BK;
    if (key0 <= q0 + 31) {
      tile(kt, key0 + BK - 1 > q0);
    } else if (kt + 1 < ntiles) {
      stage.load(kt + 1, smem + ((kt + 1) & 1) * (2 * BK * D * 2));
    }
    dma_sync();
  }
  u16* out = dq + ((size_t)(b * H + hq) * S + myq) * D;
  // T21 widened stores, as the forward's
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; g4 += 2) {
      u16x4 va, vb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        va[e] = f2bf(dqt[dt][4 * g4 + e] * scale);
        vb[e] = f2bf(dqt[dt][4 * g4 + 4 + e] * scale);
      }
      const auto a = __builtin_bit_cast(uint2, va), bb = __builtin_bit_cast(uint2, vb);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a.x, bb.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a.y, bb.y, false, false);
      const uint4 o4 = {s0[0], s1[0], s0[1], s1[1]};
      *reinterpret_cast<uint4*>(out + 32 * dt + 8 * g4 + 8 * hh) = o4;
    }
}

// ==================================================================================== host
hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }
const u16* bp(const at::Tensor& t) { return reinterpret_cast<const u16*>(t.data_ptr()); }
u16* bpm(at::Tensor& t) { return reinterpret_cast<u16*>(t.data_ptr()); }

void check_qkv(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  for (const at::Tensor* x : {&q, &k, &v})
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kBFloat16 && x->is_contiguous() && x->dim() == 4,
                "attention: q/k/v must be contiguous bf16 [B, heads, S, D] GPU tensors");
  TORCH_CHECK(q.size(3) == D && k.size(3) == D && v.size(3) == D, "attention: head dim must be 128");
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(2) == k.size(2), "attention: shape mismatch");
  TORCH_CHECK(q.size(1) % k.size(1) == 0, "attention: q heads must be a multiple of kv heads");
  TORCH_CHECK(q.size(2) % BQ == 0, "attention: sequence length must be a multiple of 128");
  TORCH_CHECK(q.size(1) * q.size(2) * D * 2 < (int64_t(1) << 31), "attention: per-batch q/dO bytes must fit the 32-bit buffer offsets");
}

// forward (fwd2); with_t: also O^T [H*D, B*S] (the o-projection's NT-layout x^T) from the epilogue
std::vector<at::Tensor> attn_fwd_impl(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                      bool with_t) {
  check_qkv(q, k, v);
  const int B = q.size(0), H = q.size(1), S = q.size(2), Hkv = k.size(1);
  auto o = at::empty({B, S, H, D}, q.options());
  auto lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  const float c = (float)(scale * 1.4426950408889634);
  at::Tensor ot;
  if (with_t) ot = at::empty({(int64_t)H * D, (int64_t)B * S}, q.options());
  hipLaunchKernelGGL(attn_fwd2_kernel, dim3(B * H, S / BQ), dim3(256), 0, cur_stream(), bp(q), bp(k), bp(v), bpm(o),
                     lse.data_ptr<float>(), H, Hkv, S, c, with_t ? bpm(ot) : nullptr);
  if (with_t) return {o, lse, ot};
  return {o, lse};
}

// {o, lse, ot}
std::vector<at::Tensor> attn_fwd_t(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale) {
  return attn_fwd_impl(q, k, v, scale, true);
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale) {
  return attn_fwd_impl(q, k, v, scale, false);
}

// backward: delta (+ -lse/c, -delta for dK/dV), dK/dV, dQ
std::vector<at::Tensor> attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                 const at::Tensor& out, const at::Tensor& lse, double scale) {
  check_qkv(q, k, v);
  const int B = q.size(0), H = q.size(1), S = q.size(2), Hkv = k.size(1);
  TORCH_CHECK(dout.is_contiguous() && out.is_contiguous() && dout.numel() == q.numel() && out.numel() == q.numel(),
              "attention bwd: dout/out must be contiguous [B, S, H, D]");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat && lse.numel() == (int64_t)B * H * S,
              "attention bwd: lse must be fp32 [B, H, S]");
  auto fopt = q.options().dtype(at::kFloat);
  auto delta = at::empty({B, H, S}, fopt), nls = at::empty({B, H, S}, fopt), ndl = at::empty({B, H, S}, fopt);
  auto dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  const int rows = B * S * H;
  const float c = (float)(scale * 1.4426950408889634);
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows + 15) / 16), dim3(256), 0, cur_stream(), bp(dout), bp(out),
                     lse.data_ptr<float>(), delta.data_ptr<float>(), nls.data_ptr<float>(), ndl.data_ptr<float>(), B, H, S,
                     1.f / c);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3(B * Hkv, S / KB), dim3(256), 0, cur_stream(), bp(q), bp(k), bp(v), bp(dout),
                     nls.data_ptr<float>(), ndl.data_ptr<float>(), bpm(dk), bpm(dv), H, Hkv, S, c, (float)scale);
  hipLaunchKernelGGL(attn_bwd_dq2n_kernel, dim3(B * H, S / BQ), dim3(256), 0, cur_stream(), bp(q), bp(k), bp(v), bp(dout),
                     lse.data_ptr<float>(), delta.data_ptr<float>(), bpm(dq), H, Hkv, S, c, (float)scale);
  return {dq, dk, dv};
}

}  // namespace gtk_attn
