// Communication shadow: what an 8-GPU data-parallel all-reduce would take from the compute of one GPU
// (VERDICT r3 next #4).
//
// During a DP backward, every completed gradient bucket starts an RCCL ring all-reduce whose kernel
// occupies N CUs (its CTAs, one per channel) for as long as the xGMI links take to move the bucket:
// each member sends and receives 2(k-1)/k of the bucket, so the collective lasts
// bytes * 2(k-1)/k / busBW.  The training GEMMs run on the remaining CUs meanwhile.  A one-GPU box
// cannot run that collective, but it can run its shadow: this kernel takes N workgroups of 256
// threads (RCCL's CTA shape), copies the bytes the collective would move through local HBM, paced
// in chunks so that the copy is spread over the collective's duration (on a node the bytes arrive
// over xGMI at the link rate, not at HBM rate), and keeps its CUs until that duration has elapsed.
// Launched on a side stream at each bucket-ready hook (parallel/dp.py comm_shadow), it reproduces the
// CU contention and the HBM traffic of the real collective, and the step-time inflation it causes is
// what the 8-GPU step would pay for its communication (profiles/r04_comm_shadow).
//
// Timing: wall_clock64() is the 100 MHz constant clock (s_memrealtime), so the pacing does not drift
// with the shader clock.  Every workgroup exits once its last chunk's deadline has passed: the loop is
// bounded by `chunks` and the deadline is finite, so the grid always drains.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstdint>

namespace gtk_shadow {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void comm_shadow_kernel(const u16x8* __restrict__ src, u16x8* __restrict__ dst,
                                                          int64_t vec_per_chunk, int chunks, int64_t ticks_per_chunk) {
  const int64_t base = (int64_t)blockIdx.x * vec_per_chunk * chunks;
  const long long t0 = wall_clock64();
  for (int c = 0; c < chunks; ++c) {
    const int64_t o = base + (int64_t)c * vec_per_chunk;
    for (int64_t i = threadIdx.x; i < vec_per_chunk; i += 256) dst[o + i] = src[o + i];
    const long long deadline = t0 + (long long)(c + 1) * ticks_per_chunk;
    while (wall_clock64() < deadline) __builtin_amdgcn_s_sleep(8);
  }
}

// Move `bytes` (rounded down to whole 16-B vectors per workgroup and chunk) from src to dst with
// `ctas` workgroups over at least `micros` microseconds.  src/dst: contiguous GPU buffers of >= bytes.
void comm_shadow(const at::Tensor& src, at::Tensor& dst, int64_t bytes, int64_t ctas, double micros) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous(), "comm_shadow: contiguous GPU buffers");
  TORCH_CHECK(ctas >= 1 && ctas <= 4096, "comm_shadow: 1..4096 workgroups");
  TORCH_CHECK(bytes >= 0 && bytes <= (int64_t)src.nbytes() && bytes <= (int64_t)dst.nbytes(), "comm_shadow: buffers too small");
  TORCH_CHECK(micros >= 0 && micros < 10e6, "comm_shadow: duration out of range");
  const int chunks = 16;
  const int64_t vec_per_chunk = bytes / 16 / ctas / chunks;
  const int64_t ticks = (int64_t)(micros * 100.0 / chunks);  // 100 MHz wall clock
  hipLaunchKernelGGL(comm_shadow_kernel, dim3((unsigned)ctas), dim3(256), 0, at::hip::getCurrentHIPStream().stream(),
                     reinterpret_cast<const u16x8*>(src.data_ptr()), reinterpret_cast<u16x8*>(dst.data_ptr()), vec_per_chunk,
                     chunks, ticks);
}

}  // namespace gtk_shadow
