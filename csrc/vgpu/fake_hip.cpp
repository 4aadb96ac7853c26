// Stand-in HIP runtime (host-only) for CPU tests of libgtk_vgpu.so.  Layered like the real one: every
// entry point initialises the stand-in ROCr (fake_hsa.cpp, linked as libhsa-runtime64.so) through
// hsa_init, device allocations come from the current GPU's global pool (hsa_amd_memory_pool_allocate),
// host allocations from the CPU pool, hipMemCreate from hsa_amd_vmem_handle_create, and a stream is
// an HSA queue on the current GPU.  Built as bin/fake_hip/libamdhip64.so so the guard's fallback
// lookup (a runtime loaded RTLD_LOCAL, found by name among the loaded objects) is exercised exactly
// as with the PyTorch wheel's bundled runtime.  The current device comes from $FAKE_HIP_DEVICE, a HIP
// ordinal: $HIP_VISIBLE_DEVICES maps it to a ROCr ordinal and the stand-in ROCr's $ROCR_VISIBLE_DEVICES
// that to a physical GPU, whose PCI address hipDeviceGetPCIBusId reports.  Each device has 64 GiB.
// hipMallocManaged returns system memory that no device pool is charged for (HMM-backed managed memory,
// ADVICE r4), which the guard has to charge at the HIP level.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_set>

extern "C" {
// the stand-in ROCr's test hooks
const char* fake_hsa_init_mask();
const char* fake_hsa_queue_mask(const hsa_queue_t* q);
uint64_t fake_hsa_gpu_pool(int gpu);
uint64_t fake_hsa_cpu_pool();
uint64_t fake_hsa_gpu_agent(int gpu);
int fake_hsa_physical(int ordinal);
int fake_hsa_visible_count();

typedef int hipError_t;
static const unsigned long long kTotal = 64ull << 30;
static const hipError_t kOk = 0, kInvalid = 1, kOom = 2;

struct hipExtent {
  size_t width, height, depth;
};
struct hipPitchedPtr {
  void* ptr;
  size_t pitch, xsize, ysize;
};

// HIP ordinal -> ROCr ordinal ($HIP_VISIBLE_DEVICES), -1 when not visible
static int rocr_ordinal(int hip) {
  const char* v = std::getenv("HIP_VISIBLE_DEVICES");
  if (!v || !*v) return hip;
  int i = 0;
  for (const char* c = v; *c; ++i) {
    char* e = nullptr;
    long o = std::strtol(c, &e, 10);
    if (e == c) break;
    if (i == hip) return (int)o;
    c = *e == ',' ? e + 1 : e;
  }
  return -1;
}

static int physical(int hip) { return fake_hsa_physical(rocr_ordinal(hip)); }

static int hip_device() {
  const char* e = std::getenv("FAKE_HIP_DEVICE");
  return e ? std::atoi(e) : 0;
}

static int cur() {  // the current device, as the physical GPU whose pool / agent serve it
  const int p = physical(hip_device());
  return p < 0 ? 0 : p;
}

static void init() { hsa_init(); }

static hipError_t status(hsa_status_t s) {
  return s == HSA_STATUS_SUCCESS ? kOk : s == HSA_STATUS_ERROR_OUT_OF_RESOURCES ? kOom : kInvalid;
}

// managed blocks handed out (hipFree must tell them from pool blocks without touching memory)
static std::mutex g_managed_mu;
static std::unordered_set<void*>& g_managed() {
  static auto* m = new std::unordered_set<void*>();  // never destroyed: frees may come from exit-time code
  return *m;
}
static bool g_managed_take(void* p) {  // forget p if it is a managed block; -> whether it was
  std::lock_guard<std::mutex> g(g_managed_mu);
  return g_managed().erase(p) != 0;
}

static hipError_t dev_alloc(void** p, size_t n) {
  init();
  if (!p) return kInvalid;
  hipError_t e = status(hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t{fake_hsa_gpu_pool(cur())}, n, 0, p));
  if (e != kOk) *p = nullptr;
  return e;
}

__attribute__((visibility("default"))) const char* fake_hip_init_mask() { return fake_hsa_init_mask(); }
__attribute__((visibility("default"))) const char* fake_hip_stream_mask(void* stream) {
  return fake_hsa_queue_mask(static_cast<const hsa_queue_t*>(stream));
}

__attribute__((visibility("default"))) hipError_t hipInit(unsigned int) {
  init();
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipGetDeviceCount(int* n) {
  init();
  if (n) *n = fake_hsa_visible_count();
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipDeviceGetPCIBusId(char* bus, int len, int dev) {
  init();
  const int p = physical(dev);
  if (!bus || len < 13 || p < 0) return kInvalid;
  std::snprintf(bus, (size_t)len, "0000:%02x:00.0", 0x05 + 0x10 * p);
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipSetDevice(int) {
  init();
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipGetDevice(int* d) {
  init();
  *d = hip_device();
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipRuntimeGetVersion(int* v) {
  init();
  if (v) *v = 70200000;
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipDeviceGetAttribute(int* v, int, int) {
  init();
  if (v) *v = 256;
  return kOk;
}

__attribute__((visibility("default"))) hipError_t hipMalloc(void** p, size_t n) { return dev_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipExtMallocWithFlags(void** p, size_t n, unsigned int) { return dev_alloc(p, n); }
static const unsigned kManagedTag = 0x6d616e67;  // "mang": system memory, freed by hipFree like device memory
__attribute__((visibility("default"))) hipError_t hipMallocManaged(void** p, size_t n, unsigned int) {
  init();
  if (!p) return kInvalid;
  // FAKE_HIP_MANAGED_IN_POOL=1: a runtime that backs managed memory with a device pool (no HMM): the
  // guard's pool hook charges it, and its HIP-level hook must not charge it again
  if (const char* v = std::getenv("FAKE_HIP_MANAGED_IN_POOL"); v && v[0] == '1') return dev_alloc(p, n);
  unsigned* b = static_cast<unsigned*>(std::malloc(32 + (n & 7)));
  if (!b) return kOom;
  b[0] = kManagedTag;
  *p = b + 4;
  std::lock_guard<std::mutex> g(g_managed_mu);
  g_managed().insert(*p);
  return kOk;
}
__attribute__((visibility("default"))) hipError_t hipMallocAsync(void** p, size_t n, void*) { return dev_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipMallocFromPoolAsync(void** p, size_t n, void*, void*) { return dev_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  const size_t pw = (w + 255) & ~(size_t)255;
  if (pitch) *pitch = pw;
  return dev_alloc(p, pw * h);
}
__attribute__((visibility("default"))) hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent ext) {
  if (!pp) return kInvalid;
  const size_t pw = (ext.width + 255) & ~(size_t)255;
  pp->pitch = pw;
  pp->xsize = ext.width;
  pp->ysize = ext.height;
  return dev_alloc(&pp->ptr, pw * ext.height * (ext.depth ? ext.depth : 1));
}
__attribute__((visibility("default"))) hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
  init();
  if (!p) return kInvalid;
  return status(hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t{fake_hsa_cpu_pool()}, n, 0, p));
}
__attribute__((visibility("default"))) hipError_t hipFree(void* p) {
  init();
  if (!p) return kOk;
  if (g_managed_take(p)) {
    std::free(static_cast<unsigned*>(p) - 4);
    return kOk;
  }
  return status(hsa_amd_memory_pool_free(p));
}
__attribute__((visibility("default"))) hipError_t hipFreeAsync(void* p, void*) { return hipFree(p); }
__attribute__((visibility("default"))) hipError_t hipHostFree(void* p) { return hipFree(p); }
__attribute__((visibility("default"))) hipError_t hipMemCreate(void** h, size_t n, const void*, unsigned long long) {
  init();
  hsa_amd_vmem_alloc_handle_t vh{0};
  hipError_t e = status(hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t{fake_hsa_gpu_pool(cur())}, n, MEMORY_TYPE_NONE, 0, &vh));
  if (h) *h = e == kOk ? reinterpret_cast<void*>(vh.handle) : nullptr;
  return e;
}
__attribute__((visibility("default"))) hipError_t hipMemRelease(void* h) {
  return status(hsa_amd_vmem_handle_release(hsa_amd_vmem_alloc_handle_t{reinterpret_cast<uint64_t>(h)}));
}
__attribute__((visibility("default"))) hipError_t hipMemGetInfo(size_t* f, size_t* t) {
  init();
  if (f) *f = kTotal;
  if (t) *t = kTotal;
  return kOk;
}

// a stream is an HSA queue on the current device (its handle is the queue's address here)
__attribute__((visibility("default"))) hipError_t hipStreamCreate(void** stream) {
  init();
  hsa_queue_t* q = nullptr;
  hipError_t e = status(hsa_queue_create(hsa_agent_t{fake_hsa_gpu_agent(cur())}, 4096, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr,
                                         0, 0, &q));
  if (stream) *stream = q;
  return e;
}
__attribute__((visibility("default"))) hipError_t hipExtStreamCreateWithCUMask(void** stream, uint32_t count, const uint32_t* mask) {
  hipError_t e = hipStreamCreate(stream);
  if (e != kOk) return e;
  return status(hsa_amd_queue_cu_set_mask(static_cast<hsa_queue_t*>(*stream), count * 32, mask));  // words -> bits
}
__attribute__((visibility("default"))) hipError_t hipStreamDestroy(void* stream) {
  return status(hsa_queue_destroy(static_cast<hsa_queue_t*>(stream)));
}
}
