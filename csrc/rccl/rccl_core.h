// RCCL all-reduce placement validator core (shared by the `_rccl` pybind module and the
// standalone `rccl_allreduce_bench` binary).
//
// Reference: nothing — the reference design stops at pod annotations (design.md:223-246); Gaia's
// only workload check is a 2-GPU MNIST run (paper p.7 Exp. 6).  BASELINE.json's north-star metric
// asks for "RCCL all-reduce bus GB/s on the scheduler-chosen k-GPU subset"; SURVEY.md §2.C C1 and
// §3.5 specify this component: ncclCommInitAll over the chosen device list (single process) or
// ncclCommInitRank (one process per GPU), bf16/fp32 sum, algBW = bytes/t, busBW = algBW*2(k-1)/k
// (nccl-tests convention), with an exact correctness check.
//
// Correctness data: rank r contributes (r+1)*((i%7)+1); every partial sum stays < 256 so bf16
// represents it exactly and the reduced value must equal ((i%7)+1)*k(k+1)/2 bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#define RCCL_HIP_CHECK(expr)                                                                     \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess)                                                                        \
      throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                       \
  } while (0)

#define NCCL_CHECK(expr)                                                                          \
  do {                                                                                            \
    ncclResult_t _r = (expr);                                                                     \
    if (_r != ncclSuccess)                                                                        \
      throw std::runtime_error(std::string(#expr " failed: ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                        \
  } while (0)

namespace gtk {

inline ncclDataType_t parse_dtype(const std::string& s, size_t* elem) {
  if (s == "bf16" || s == "bfloat16") {
    *elem = 2;
    return ncclBfloat16;
  }
  if (s == "fp16" || s == "half" || s == "float16") {
    *elem = 2;
    return ncclFloat16;
  }
  if (s == "fp32" || s == "float" || s == "float32") {
    *elem = 4;
    return ncclFloat32;
  }
  throw std::invalid_argument("dtype must be bf16|fp16|fp32");
}

inline double bus_factor(int k) { return k > 1 ? 2.0 * (k - 1) / k : 0.0; }

// ---------------------------------------------------------------------------------- kernels
__global__ void gtk_fill_kernel(void* buf, size_t count, int dtype_code, int rank) {
  const float scale = (float)(rank + 1);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    float v = scale * (float)((i % 7) + 1);
    if (dtype_code == 0) {
      __bf16 b = (__bf16)v;
      reinterpret_cast<__bf16*>(buf)[i] = b;
    } else if (dtype_code == 1) {
      reinterpret_cast<_Float16*>(buf)[i] = (_Float16)v;
    } else {
      reinterpret_cast<float*>(buf)[i] = v;
    }
  }
}

__global__ void gtk_check_kernel(const void* buf, size_t count, int dtype_code, int nranks,
                                 unsigned long long* bad) {
  const float tri = (float)(nranks * (nranks + 1) / 2);
  unsigned long long local = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    float want = tri * (float)((i % 7) + 1);
    float got;
    if (dtype_code == 0)
      got = (float)reinterpret_cast<const __bf16*>(buf)[i];
    else if (dtype_code == 1)
      got = (float)reinterpret_cast<const _Float16*>(buf)[i];
    else
      got = reinterpret_cast<const float*>(buf)[i];
    local += (got != want);
  }
  if (local) atomicAdd(bad, local);
}

inline int dtype_code(ncclDataType_t t) { return t == ncclBfloat16 ? 0 : (t == ncclFloat16 ? 1 : 2); }

// ---------------------------------------------------------------------------------- one rank
// One communicator member on one device with persistent send/recv buffers.
struct RankState {
  int device = -1, rank = 0, nranks = 1;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  void* send = nullptr;
  void* recv = nullptr;
  size_t cap_bytes = 0;

  void set_device() const { RCCL_HIP_CHECK(hipSetDevice(device)); }

  void ensure(size_t bytes) {
    set_device();
    if (!stream) RCCL_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    if (bytes <= cap_bytes) return;
    if (send) RCCL_HIP_CHECK(hipFree(send));
    if (recv) RCCL_HIP_CHECK(hipFree(recv));
    send = recv = nullptr;
    RCCL_HIP_CHECK(hipMalloc(&send, bytes));
    RCCL_HIP_CHECK(hipMalloc(&recv, bytes));
    cap_bytes = bytes;
  }

  void fill(size_t count, ncclDataType_t t) {
    set_device();
    hipLaunchKernelGGL(gtk_fill_kernel, dim3(1024), dim3(256), 0, stream, send, count, dtype_code(t), rank);
    RCCL_HIP_CHECK(hipGetLastError());
  }

  unsigned long long check(size_t count, ncclDataType_t t, bool inplace) {
    set_device();
    unsigned long long* d_bad = nullptr;
    RCCL_HIP_CHECK(hipMalloc(&d_bad, sizeof(unsigned long long)));
    RCCL_HIP_CHECK(hipMemsetAsync(d_bad, 0, sizeof(unsigned long long), stream));
    hipLaunchKernelGGL(gtk_check_kernel, dim3(1024), dim3(256), 0, stream, inplace ? send : recv, count, dtype_code(t),
                       nranks, d_bad);
    RCCL_HIP_CHECK(hipGetLastError());
    unsigned long long bad = 0;
    RCCL_HIP_CHECK(hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, stream));
    RCCL_HIP_CHECK(hipStreamSynchronize(stream));
    RCCL_HIP_CHECK(hipFree(d_bad));
    return bad;
  }

  void allreduce(size_t count, ncclDataType_t t, bool inplace) {
    NCCL_CHECK(ncclAllReduce(send, inplace ? send : recv, count, t, ncclSum, comm, stream));
  }

  void release() {
    if (comm) {
      (void)hipSetDevice(device);
      (void)ncclCommDestroy(comm);
      comm = nullptr;
    }
    if (send) (void)hipFree(send);
    if (recv) (void)hipFree(recv);
    send = recv = nullptr;
    cap_bytes = 0;
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

struct SweepPoint {
  size_t bytes = 0;
  size_t count = 0;
  double time_us = 0, algbw = 0, busbw = 0;
  unsigned long long wrong = 0;
};

// ---------------------------------------------------------------------------------- single process
// All k devices in this process (ncclCommInitAll + ncclGroupStart/End), the SURVEY §3.5 validator.
class LocalGroup {
 public:
  explicit LocalGroup(const std::vector<int>& devs) : ranks_(devs.size()) {
    if (devs.empty()) throw std::invalid_argument("empty device list");
    std::vector<ncclComm_t> comms(devs.size());
    std::vector<int> dl(devs.begin(), devs.end());
    NCCL_CHECK(ncclCommInitAll(comms.data(), (int)devs.size(), dl.data()));
    for (size_t i = 0; i < devs.size(); ++i) {
      ranks_[i].device = devs[i];
      ranks_[i].rank = (int)i;
      ranks_[i].nranks = (int)devs.size();
      ranks_[i].comm = comms[i];
    }
  }
  ~LocalGroup() {
    for (auto& r : ranks_) r.release();
  }
  LocalGroup(const LocalGroup&) = delete;
  LocalGroup& operator=(const LocalGroup&) = delete;

  SweepPoint run(size_t bytes, const std::string& dtype, int iters, int warmup, bool inplace, bool check) {
    size_t elem = 0;
    ncclDataType_t t = parse_dtype(dtype, &elem);
    const size_t count = std::max<size_t>(1, bytes / elem);
    bytes = count * elem;
    for (auto& r : ranks_) r.ensure(bytes);
    SweepPoint p;
    p.bytes = bytes;
    p.count = count;
    if (check) {
      for (auto& r : ranks_) r.fill(count, t);
      launch_all(count, t, inplace);
      sync_all();
      for (auto& r : ranks_) p.wrong += r.check(count, t, inplace);
    }
    for (int i = 0; i < warmup; ++i) launch_all(count, t, inplace);
    sync_all();
    std::vector<hipEvent_t> e0(ranks_.size()), e1(ranks_.size());
    for (size_t i = 0; i < ranks_.size(); ++i) {
      ranks_[i].set_device();
      RCCL_HIP_CHECK(hipEventCreate(&e0[i]));
      RCCL_HIP_CHECK(hipEventCreate(&e1[i]));
      RCCL_HIP_CHECK(hipEventRecord(e0[i], ranks_[i].stream));
    }
    for (int i = 0; i < iters; ++i) launch_all(count, t, inplace);
    float worst = 0.f;
    for (size_t i = 0; i < ranks_.size(); ++i) {
      ranks_[i].set_device();
      RCCL_HIP_CHECK(hipEventRecord(e1[i], ranks_[i].stream));
    }
    for (size_t i = 0; i < ranks_.size(); ++i) {
      ranks_[i].set_device();
      RCCL_HIP_CHECK(hipEventSynchronize(e1[i]));
      float ms = 0.f;
      RCCL_HIP_CHECK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      worst = std::max(worst, ms);
      (void)hipEventDestroy(e0[i]);
      (void)hipEventDestroy(e1[i]);
    }
    p.time_us = worst * 1e3 / std::max(1, iters);
    p.algbw = (double)bytes / (p.time_us * 1e-6) / 1e9;
    p.busbw = p.algbw * bus_factor((int)ranks_.size());
    return p;
  }

  size_t size() const { return ranks_.size(); }

 private:
  void launch_all(size_t count, ncclDataType_t t, bool inplace) {
    NCCL_CHECK(ncclGroupStart());
    for (auto& r : ranks_) {
      r.set_device();
      r.allreduce(count, t, inplace);
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void sync_all() {
    for (auto& r : ranks_) {
      r.set_device();
      RCCL_HIP_CHECK(hipStreamSynchronize(r.stream));
    }
  }
  std::vector<RankState> ranks_;
};

inline std::vector<size_t> size_sweep(size_t min_bytes, size_t max_bytes, int factor) {
  std::vector<size_t> out;
  factor = std::max(2, factor);
  for (size_t b = std::max<size_t>(min_bytes, 4); b <= max_bytes; b *= (size_t)factor) {
    out.push_back(b);
    if (b > max_bytes / (size_t)factor) break;
  }
  return out;
}

}  // namespace gtk
