// Stand-in ROCr runtime (host-only) for CPU tests of libgtk_vgpu.so, built as
// bin/fake_hip/libhsa-runtime64.so and linked by the stand-in HIP runtime (fake_hip.cpp) the way the
// real libamdhip64 links libhsa-runtime64.  It models what the guard relies on:
//   * hsa_init reads HSA_CU_MASK once, as ROCr does (fake_hsa_init_mask() returns what it read);
//   * agents: a CPU agent first, then two GPU agents with 256 CUs each, physical GPU p at PCI address
//     0000:(05 + 0x10 p):00.0 (HSA_AMD_AGENT_INFO_BDFID / _DOMAIN); $ROCR_VISIBLE_DEVICES ("1,0", "1")
//     selects and orders them as ROCr does, so ordinals need not be physical indices; every agent has
//     one global memory pool; allocations are tiny host blocks (the size is bookkept);
//   * queues: a created queue starts with the CU mask HSA_CU_MASK gave its GPU at hsa_init (all CUs
//     when none), hsa_amd_queue_cu_set_mask replaces it; fake_hsa_queue_mask(q) renders the mask
//     a queue runs with as a CU list ("0-63").
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kGpus = 2;
constexpr int kCus = 256;
constexpr uint64_t kCpuAgent = 0x1000, kGpuAgent0 = 0x2000;
constexpr uint64_t kCpuPool = 0x3000, kGpuPool0 = 0x4000;

std::mutex g_mu;
bool g_inited = false;
char g_init_mask[4096] = "(never initialised)";
std::vector<uint32_t> g_env_bits[kGpus];  // HSA_CU_MASK as read at hsa_init, by ordinal
std::vector<int> g_visible;                // ordinal -> physical GPU ($ROCR_VISIBLE_DEVICES at hsa_init)

void parse_visible() {
  g_visible.clear();
  const char* v = std::getenv("ROCR_VISIBLE_DEVICES");
  if (!v || !*v) {
    for (int p = 0; p < kGpus; ++p) g_visible.push_back(p);
    return;
  }
  for (const char* c = v; *c;) {
    char* e = nullptr;
    long p = std::strtol(c, &e, 10);
    if (e == c) break;
    if (p >= 0 && p < kGpus) g_visible.push_back((int)p);
    c = *e == ',' ? e + 1 : e;
  }
}

int ordinal_of(int phys) {
  for (size_t o = 0; o < g_visible.size(); ++o)
    if (g_visible[o] == phys) return (int)o;
  return -1;
}
struct FakeQueue {
  hsa_queue_t q;
  int gpu;
  std::vector<uint32_t> mask;
};
std::unordered_map<const hsa_queue_t*, FakeQueue*> g_queues;
std::string g_last_render;

std::vector<uint32_t> all_cus() { return std::vector<uint32_t>(kCus / 32, 0xffffffffu); }

void parse_env_mask(const char* v) {
  for (auto& b : g_env_bits) b.clear();
  if (!v) return;
  std::string s(v);
  size_t i = 0;
  while (i < s.size()) {
    size_t end = s.find(';', i);
    if (end == std::string::npos) end = s.size();
    std::string part = s.substr(i, end - i);
    i = end + 1;
    size_t colon = part.find(':');
    if (colon == std::string::npos) continue;
    int dev = std::atoi(part.c_str());
    if (dev < 0 || dev >= kGpus) continue;
    std::vector<uint32_t> bits(kCus / 32, 0u);
    const char* c = part.c_str() + colon + 1;
    while (*c) {
      char* e = nullptr;
      long a = std::strtol(c, &e, 10);
      if (e == c) break;
      long b = a;
      c = e;
      if (*c == '-') {
        b = std::strtol(c + 1, &e, 10);
        c = e;
      }
      for (long cu = a; cu <= b && cu < kCus; ++cu) bits[cu / 32] |= 1u << (cu % 32);
      if (*c == ',') ++c;
    }
    g_env_bits[dev] = bits;
  }
}

std::string render(const std::vector<uint32_t>& bits) {
  std::string out;
  int cu = 0;
  const int n = (int)bits.size() * 32;
  while (cu < n) {
    if (!(bits[cu / 32] >> (cu % 32) & 1u)) {
      ++cu;
      continue;
    }
    int a = cu;
    while (cu + 1 < n && (bits[(cu + 1) / 32] >> ((cu + 1) % 32) & 1u)) ++cu;
    if (!out.empty()) out += ",";
    out += a == cu ? std::to_string(a) : std::to_string(a) + "-" + std::to_string(cu);
    ++cu;
  }
  return out;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) const char* fake_hsa_init_mask() { return g_init_mask; }

__attribute__((visibility("default"))) const char* fake_hsa_queue_mask(const hsa_queue_t* q) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_queues.find(q);
  g_last_render = it == g_queues.end() ? "(unknown queue)" : render(it->second->mask);
  return g_last_render.c_str();
}

__attribute__((visibility("default"))) hsa_status_t hsa_init() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_inited) return HSA_STATUS_SUCCESS;
  g_inited = true;
  parse_visible();
  const char* m = std::getenv("HSA_CU_MASK");
  std::strncpy(g_init_mask, m ? m : "", sizeof(g_init_mask) - 1);
  parse_env_mask(m);
  return HSA_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) hsa_status_t hsa_iterate_agents(hsa_status_t (*cb)(hsa_agent_t, void*), void* data) {
  if (!g_inited) return HSA_STATUS_ERROR_NOT_INITIALIZED;  // as ROCr before hsa_init
  hsa_agent_t a{kCpuAgent};
  hsa_status_t e = cb(a, data);
  for (size_t o = 0; o < g_visible.size() && e == HSA_STATUS_SUCCESS; ++o)
    e = cb(hsa_agent_t{kGpuAgent0 + (uint64_t)g_visible[o]}, data);
  return e == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : e;
}

__attribute__((visibility("default"))) hsa_status_t hsa_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  const bool cpu = agent.handle == kCpuAgent;
  if (attr == HSA_AGENT_INFO_DEVICE) {
    *static_cast<hsa_device_type_t*>(value) = cpu ? HSA_DEVICE_TYPE_CPU : HSA_DEVICE_TYPE_GPU;
    return HSA_STATUS_SUCCESS;
  }
  if ((int)attr == (int)HSA_AMD_AGENT_INFO_BDFID && !cpu) {  // bus << 8 | device << 3 | function
    *static_cast<uint32_t*>(value) = (uint32_t)(0x05 + 0x10 * (int)(agent.handle - kGpuAgent0)) << 8;
    return HSA_STATUS_SUCCESS;
  }
  if ((int)attr == (int)HSA_AMD_AGENT_INFO_DOMAIN && !cpu) {
    *static_cast<uint32_t*>(value) = 0;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}

// ROCr ordinal -> physical GPU (for the stand-in HIP runtime's device numbering); -1 when not visible
__attribute__((visibility("default"))) int fake_hsa_physical(int ordinal) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_inited) parse_visible();
  return ordinal >= 0 && ordinal < (int)g_visible.size() ? g_visible[ordinal] : -1;
}
__attribute__((visibility("default"))) int fake_hsa_visible_count() {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_inited) parse_visible();
  return (int)g_visible.size();
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_agent_iterate_memory_pools(
    hsa_agent_t agent, hsa_status_t (*cb)(hsa_amd_memory_pool_t, void*), void* data) {
  const uint64_t pool = agent.handle == kCpuAgent ? kCpuPool : kGpuPool0 + (agent.handle - kGpuAgent0);
  hsa_status_t e = cb(hsa_amd_memory_pool_t{pool}, data);
  return e == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : e;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_get_info(hsa_amd_memory_pool_t pool,
                                                                                  hsa_amd_memory_pool_info_t attr, void* value) {
  if (attr == HSA_AMD_MEMORY_POOL_INFO_SEGMENT) {
    *static_cast<hsa_amd_segment_t*>(value) = HSA_AMD_SEGMENT_GLOBAL;
    return HSA_STATUS_SUCCESS;
  }
  if (attr == HSA_AMD_MEMORY_POOL_INFO_LOCATION) {
    *static_cast<hsa_amd_memory_pool_location_t*>(value) =
        pool.handle == kCpuPool ? HSA_AMD_MEMORY_POOL_LOCATION_CPU : HSA_AMD_MEMORY_POOL_LOCATION_GPU;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}

// pool handles the stand-in HIP runtime allocates from
__attribute__((visibility("default"))) uint64_t fake_hsa_gpu_pool(int gpu) { return kGpuPool0 + (uint64_t)gpu; }
__attribute__((visibility("default"))) uint64_t fake_hsa_cpu_pool() { return kCpuPool; }
__attribute__((visibility("default"))) uint64_t fake_hsa_gpu_agent(int gpu) { return kGpuAgent0 + (uint64_t)gpu; }

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t, size_t size, uint32_t,
                                                                                  void** ptr) {
  if (!ptr) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  *ptr = std::malloc(16 + (size & 7));  // distinct pointers; the size itself is never touched
  return *ptr ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR_OUT_OF_RESOURCES;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  std::free(ptr);
  return HSA_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t, size_t size,
                                                                                hsa_amd_memory_type_t, uint64_t,
                                                                                hsa_amd_vmem_alloc_handle_t* h) {
  if (!h) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  h->handle = reinterpret_cast<uint64_t>(std::malloc(16 + (size & 7)));
  return h->handle ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR_OUT_OF_RESOURCES;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_vmem_handle_release(hsa_amd_vmem_alloc_handle_t h) {
  std::free(reinterpret_cast<void*>(h.handle));
  return HSA_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t, hsa_queue_type32_t,
                                                                      void (*)(hsa_status_t, hsa_queue_t*, void*), void*,
                                                                      uint32_t, uint32_t, hsa_queue_t** queue) {
  if (!queue || agent.handle < kGpuAgent0 || agent.handle >= kGpuAgent0 + kGpus) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(g_mu);
  FakeQueue* fq = new FakeQueue();
  std::memset(&fq->q, 0, sizeof(fq->q));
  fq->gpu = (int)(agent.handle - kGpuAgent0);
  const int ord = ordinal_of(fq->gpu);  // HSA_CU_MASK names ordinals, not physical GPUs
  fq->mask = (ord < 0 || g_env_bits[ord].empty()) ? all_cus() : g_env_bits[ord];
  g_queues[&fq->q] = fq;
  *queue = &fq->q;
  return HSA_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_destroy(hsa_queue_t* q) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_queues.find(q);
  if (it == g_queues.end()) return HSA_STATUS_ERROR_INVALID_QUEUE;
  delete it->second;
  g_queues.erase(it);
  return HSA_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* q, uint32_t nbits,
                                                                               const uint32_t* mask) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_queues.find(q);
  if (it == g_queues.end() || !mask || nbits % 32) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  std::vector<uint32_t> m(kCus / 32, 0u);
  for (uint32_t w = 0; w < nbits / 32 && w < m.size(); ++w) m[w] = mask[w];
  it->second->mask = m;
  return HSA_STATUS_SUCCESS;
}
}
