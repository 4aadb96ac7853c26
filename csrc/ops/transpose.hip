// bf16 2-D transpose for the Llama workload's backward GEMMs.
//
// hipBLASLt runs the "NT" layout (both operands contiguous along the reduction dimension, i.e. the
// forward GEMM's layout) 10-40 % faster than the NN layout of dgrad (dx = dy W) and the TN layout of
// wgrad (dW = dy^T x) at the Llama-3-8B shapes (bench/gemm_layout_bench.py,
// profiles/r01_llama/gemm_layout.log).  Getting an operand into NT layout costs one transpose, which
// pays only when it runs near HBM speed; torch's strided copy runs at ~0.25 TB/s on [16384, 128256]
// (8.5 ms), so the workload uses this kernel instead.
//
// Tile 64x64 bf16 per 256-thread block (4 wave64):
//   load : thread t reads 16 B (8 columns) of rows t/8 and t/8+32 -> 8 lanes cover one 128-B row
//          segment, a wave 8 rows;
//   LDS  : [64 rows][8 vectors of 16 B], vector v of row r stored at v ^ ((r>>3)&7) (XOR swizzle);
//   store: thread t gathers 8 consecutive rows r = 8p..8p+7 of one column c (8 ds_read_u16), packs
//          them into 16 B and writes out[c][8p..8p+7].  In one instruction a wave's lanes take 8
//          columns x 8 row-groups; the swizzle puts the 8 row-groups on 8 different 16-B slots, so
//          the 64 lanes touch 32 distinct banks (lane pairs share a dword): no conflicts.
// R and C must be multiples of 64; multiples of 128 (all Llama-3 dims) take the 128x128 kernel below.
// Other shapes take torch's copy.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>

namespace gtk_xpose {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

constexpr int kTile = 64;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const u16* __restrict__ x, u16* __restrict__ y, int R, int C) {
  __shared__ u16x8 tile[kTile][8];
  const int t = threadIdx.x;
  const size_t r0 = (size_t)blockIdx.y * kTile, c0 = (size_t)blockIdx.x * kTile;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (t >> 3) + 32 * i, v = t & 7;
    tile[r][v ^ ((r >> 3) & 7)] = *reinterpret_cast<const u16x8*>(x + (r0 + r) * C + c0 + 8 * v);
  }
  __syncthreads();
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i;
    const int c = idx >> 3, p = idx & 7;
    const int pv = (c >> 3) ^ p;  // ((r >> 3) & 7) == p for every r in 8p..8p+7
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[(8 * p + j) * 64 + pv * 8 + (c & 7)];
    *reinterpret_cast<u16x8*>(y + (c0 + c) * R + r0 + 8 * p) = o;
  }
}

// 128x128 tile per 256-thread block (the path for every Llama-3 shape: all dims are multiples of
// 128).  The 64x64 tile reads 128-B row segments and keeps only 2 x 16 B per thread in flight, so it
// is latency bound at ~4.2 TB/s (profiles/r01_xpose).  Here each thread issues 8 independent 16-B
// loads before touching LDS, input row segments are 256 B and output row segments 256 B.
//   LDS  : [128 rows][16 vectors], vector v of row r at slot v ^ ((r>>3)&15): 32 KiB.
//   store: output row c (input column), vector p = input rows 8p..8p+7.  16 lanes write one 256-B
//          output row segment, a wave 4 of them.  ds_read_u16 banks like ds_read_b32 (two groups
//          of 32 lanes, dword mod 32), so the lanes are ordered to give each 32-lane group 8 p
//          values x 4 columns: slots (c>>3) ^ p are 8 distinct 4-dword groups, the 4 columns two
//          dwords of each (lane pairs share one): no bank conflicts.
constexpr int kBig = 128;

__global__ __launch_bounds__(256) void transpose128_bf16_kernel(const u16* __restrict__ x, u16* __restrict__ y, int R,
                                                                int C) {
  __shared__ u16x8 tile[kBig][16];
  const int t = threadIdx.x;
  const size_t r0 = (size_t)blockIdx.y * kBig, c0 = (size_t)blockIdx.x * kBig;
  const int v = t & 15;
  u16x8 in[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) in[i] = *reinterpret_cast<const u16x8*>(x + (r0 + (t >> 4) + 16 * i) * C + c0 + 8 * v);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = (t >> 4) + 16 * i;
    tile[r][v ^ ((r >> 3) & 15)] = in[i];
  }
  __syncthreads();
  const u16* lds = reinterpret_cast<const u16*>(&tile[0][0]);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = t + 256 * i, lane = idx & 63;
    const int c = 4 * (idx >> 6) + ((lane >> 3) & 3), p = (lane & 7) + 8 * (lane >> 5);
    const int slot = (c >> 3) ^ p;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = lds[(8 * p + j) * kBig + slot * 8 + (c & 7)];
    *reinterpret_cast<u16x8*>(y + (c0 + c) * R + r0 + 8 * p) = o;
  }
}

// x [R, C] -> y [C, R] into a caller-provided contiguous buffer (the persistent W^T of the NT layout)
void transpose_bf16_out(const at::Tensor& x, at::Tensor& y) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2,
              "transpose_bf16: x must be a contiguous 2-D bf16 GPU tensor");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.dim() == 2 && y.size(0) == C &&
                  y.size(1) == R,
              "transpose_bf16_out: y must be a contiguous [C, R] bf16 GPU tensor");
  TORCH_CHECK(R % kTile == 0 && C % kTile == 0, "transpose_bf16: both dims must be multiples of 64");
  TORCH_CHECK(R / kTile <= 65535, "transpose_bf16: too many rows for the grid");
  if (R == 0 || C == 0) return;
  if (R % kBig == 0 && C % kBig == 0) {
    hipLaunchKernelGGL(transpose128_bf16_kernel, dim3((unsigned)(C / kBig), (unsigned)(R / kBig)), dim3(256), 0,
                       at::hip::getCurrentHIPStream().stream(), reinterpret_cast<const u16*>(x.data_ptr()),
                       reinterpret_cast<u16*>(y.data_ptr()), (int)R, (int)C);
    return;
  }
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)(C / kTile), (unsigned)(R / kTile)), dim3(256), 0,
                     at::hip::getCurrentHIPStream().stream(), reinterpret_cast<const u16*>(x.data_ptr()),
                     reinterpret_cast<u16*>(y.data_ptr()), (int)R, (int)C);
}

at::Tensor transpose_bf16(const at::Tensor& x) {
  TORCH_CHECK(x.dim() == 2, "transpose_bf16: x must be 2-D");
  auto y = at::empty({x.size(1), x.size(0)}, x.options());
  transpose_bf16_out(x, y);
  return y;
}

}  // namespace gtk_xpose
