// Stand-in HIP runtime (host-only) for CPU tests of libgtk_vgpu.so: the allocation entry points the
// guard intercepts, backed by tiny host allocations (the requested size is only bookkept), a current
// device from $FAKE_HIP_DEVICE and a 64 GiB device.  Built as bin/fake_hip/libamdhip64.so so the
// guard's fallback lookup (a runtime loaded RTLD_LOCAL, found by name among the loaded objects) is
// exercised exactly as with the PyTorch wheel's bundled runtime.  Like ROCr, it reads HSA_CU_MASK
// once, at the first call into it (its "initialisation"); fake_hip_init_mask() returns what it read.
#include <cstdlib>
#include <cstring>

extern "C" {

typedef int hipError_t;
static const unsigned long long kTotal = 64ull << 30;
static char g_init_mask[4096] = "(never initialised)";
static int g_inited = 0;

static void fake_init() {
  if (g_inited) return;
  g_inited = 1;
  const char* m = std::getenv("HSA_CU_MASK");
  std::strncpy(g_init_mask, m ? m : "", sizeof(g_init_mask) - 1);
}

__attribute__((visibility("default"))) const char* fake_hip_init_mask() { return g_init_mask; }

__attribute__((visibility("default"))) hipError_t hipInit(unsigned int) {
  fake_init();
  return 0;
}
__attribute__((visibility("default"))) hipError_t hipGetDeviceCount(int* n) {
  fake_init();
  if (n) *n = 2;
  return 0;
}
__attribute__((visibility("default"))) hipError_t hipSetDevice(int) {
  fake_init();
  return 0;
}

__attribute__((visibility("default"))) hipError_t hipGetDevice(int* d) {
  fake_init();
  const char* e = std::getenv("FAKE_HIP_DEVICE");
  *d = e ? std::atoi(e) : 0;
  return 0;
}

static hipError_t fake_alloc(void** p, size_t n) {
  fake_init();
  if (!p) return 1;
  *p = std::malloc(16 + (n & 7));  // distinct pointers; the size itself is never touched
  return *p ? 0 : 2;
}

__attribute__((visibility("default"))) hipError_t hipMalloc(void** p, size_t n) { return fake_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipExtMallocWithFlags(void** p, size_t n, unsigned int) {
  return fake_alloc(p, n);
}
__attribute__((visibility("default"))) hipError_t hipMallocManaged(void** p, size_t n, unsigned int) { return fake_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipMallocAsync(void** p, size_t n, void*) { return fake_alloc(p, n); }
__attribute__((visibility("default"))) hipError_t hipMallocFromPoolAsync(void** p, size_t n, void*, void*) {
  return fake_alloc(p, n);
}
__attribute__((visibility("default"))) hipError_t hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  if (pitch) *pitch = (w + 255) & ~(size_t)255;
  return fake_alloc(p, w * h);
}
__attribute__((visibility("default"))) hipError_t hipFree(void* p) {
  std::free(p);
  return 0;
}
__attribute__((visibility("default"))) hipError_t hipFreeAsync(void* p, void*) {
  std::free(p);
  return 0;
}
__attribute__((visibility("default"))) hipError_t hipMemCreate(void** h, size_t n, const void*, unsigned long long) {
  return fake_alloc(h, n);
}
__attribute__((visibility("default"))) hipError_t hipMemRelease(void* h) {
  std::free(h);
  return 0;
}
__attribute__((visibility("default"))) hipError_t hipMemGetInfo(size_t* f, size_t* t) {
  fake_init();
  if (f) *f = kTotal;
  if (t) *t = kTotal;
  return 0;
}
}
