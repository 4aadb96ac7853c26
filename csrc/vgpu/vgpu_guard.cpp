// libgtk_vgpu.so — the container-side tier of a time-sliced GPU share (Gaia's two-tier vGPU).
//
// Reference: the Gaia paper (p.3 §III.A "GPU resource virtualization") splits a GPU into vGPUs in
// its device plugin and enforces each vGPU's limits inside the container by intercepting the GPU API
// (GaiaGPU's interception library).  On MI355X the device plugin already gives a pod holding part of
// a GPU its slices' compute units (HSA_CU_MASK, topology/shares.py) and its HBM share
// (GTK_GPU_FRACTION); both were cooperative: a container could rewrite its environment, and only the
// framework's own training entry point capped its allocator.  This library, which Allocate mounts
// into the container and preloads (deviceplugin/plugin.py, --share-guard), makes them hold for any
// HIP program in the pod.  It enforces at the ROCr (HSA) runtime, the layer every HIP entry point
// ends in, not at a list of HIP calls:
//
//   * HBM: every device-memory pool allocation of the process (hsa_amd_memory_pool_allocate on a
//     GPU's global pool, hsa_amd_vmem_handle_create) is counted against the device's limit and
//     refused with HSA_STATUS_ERROR_OUT_OF_RESOURCES beyond it (HIP turns that into
//     hipErrorOutOfMemory).  So hipMalloc, hipMallocPitch/3D/Array, hipMallocAsync pools, hipMemCreate
//     and the runtime's own device allocations are all charged, once.  Host pools are not counted.
//     hipMallocManaged is the one HIP allocation that need not reach a device pool (with HMM the
//     runtime backs it with system memory that migrates into HBM on first touch): it is charged at
//     the HIP level, against the current device, in full, when the runtime did not already charge it
//     through a pool (and released by hipFree).  hipMemGetInfo reports the share as the device's
//     total, so caching allocators size themselves to it.
//   * CUs: HSA_CU_MASK is set from the mounted config in the constructor (before main), and set back
//     again in hsa_init, which every HIP program passes through whatever its first HIP call is, in
//     case the program rewrote it meanwhile.  Independently of the environment, every queue the
//     runtime creates (hsa_queue_create) gets the share's mask applied, and a program's own
//     hsa_amd_queue_cu_set_mask (hipExtStreamCreateWithCUMask) is intersected with it: no queue of the
//     process can run on a CU outside the share.
//
// The config is the read-only file the plugin mounts at /etc/gtk-vgpu.conf.  When that file exists it
// is the only one read: $GTK_VGPU_CONFIG (which the pod spec could override) is honoured only where
// no config is mounted (tests, hand-run jobs).  Format:
//     hbm_limit_bdf <pci address> <bytes> [<fallback ordinal>]   e.g. hbm_limit_bdf 0000:05:00.0 103079215104 0
//     cu_mask_bdf <pci address> <cu list> [<fallback ordinal>]   e.g. cu_mask_bdf 0000:05:00.0 0-127 0
//     hbm_limit <ordinal> <bytes>             (hand-run jobs) ROCr enumeration order
//     cu_mask <HSA_CU_MASK value>             (hand-run jobs) ROCr ordinals
//     acct <path>                  (optional) pod-wide accounting file, shared read-write
// The plugin writes the PCI-address forms: a device's ordinal depends on $ROCR_VISIBLE_DEVICES /
// $HIP_VISIBLE_DEVICES, which the pod can set.  Addresses are resolved to ROCr ordinals
// once the runtime has enumerated its agents (HSA_AMD_AGENT_INFO_DOMAIN / _BDFID), and HIP's device
// numbers are mapped through hipDeviceGetPCIBusId, so a share holds whatever the process renumbers.
// With address-keyed masks the environment mask is cleared instead of set (ROCr reads it before any
// agent can be named by address); the per-queue mask below is then the enforcement.
// No file: the library is inert (pure pass-through).  Without ``acct`` the limit holds per process.
// With it, every process of the pod that maps the file draws from one budget: the file is a table of
// per-process slots (bytes in use per device); a process owns its slot by holding an fcntl write lock
// on the slot's first byte, so the kernel drops a crashed process's usage with its lock — whatever PID
// namespace the pod's containers live in — and the next process reuses the slot.
//
// The real entry points are found with dlsym(RTLD_NEXT); when the runtime was loaded RTLD_LOCAL (the
// PyTorch wheel's bundled libamdhip64 and its libhsa-runtime64, brought in by Python's extension
// loader) RTLD_NEXT does not see it, so the loaded objects are searched for the library by name and it
// is re-opened RTLD_NOLOAD.  Host-only C++ (g++): the HSA headers for the types, no device code, no
// link against any ROCm library.
#include <dlfcn.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <link.h>
#include <pthread.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#ifndef GTK_VGPU_FIXED_CONF
#define GTK_VGPU_FIXED_CONF "/etc/gtk-vgpu.conf"
#endif

namespace {

typedef int hipError_t;  // enum hipError_t: int-sized
constexpr hipError_t kSuccess = 0;
constexpr int kMaxDev = 64;

// pod-wide accounting table (the `acct` file)
constexpr int kSlots = 128;
constexpr uint64_t kMagic = 0x67746b7667707531ull;  // "gtkvgpu1"
struct Slot {
  int32_t pid;
  int32_t reserved;
  int64_t used[kMaxDev];
};
struct Table {
  uint64_t magic;
  uint64_t nslots;
  Slot slot[kSlots];
};

struct State {
  std::mutex mu;
  bool active = false;
  int acct_fd = -1;          // shared accounting file (pod-wide budget), -1 = per process
  Table* table = nullptr;
  int mine = -1;             // this process's slot
  pid_t mine_pid = 0;        // the process that claimed `mine` (a forked child claims its own)
  std::atomic<long long> limit[kMaxDev];  // bytes; < 0 = no limit (atomic: resolved lazily, read unlocked)
  long long used[kMaxDev];
  std::unordered_map<void*, std::pair<int, size_t>> ptrs;                  // pool allocations
  std::unordered_map<uint64_t, std::pair<int, size_t>> handles;            // vmem handles
  std::string cu_mask;                                                     // HSA_CU_MASK value
  std::vector<std::vector<uint32_t>> mask_bits;                            // per ordinal; empty = all CUs
  std::unordered_map<const hsa_queue_t*, int> queues;                      // queue -> GPU ordinal
  std::unordered_map<void*, std::pair<int, size_t>> managed;               // hipMallocManaged charges
  struct BdfLimit {
    uint32_t addr;
    long long bytes;
    int fallback;  // ROCr ordinal to apply it to when no agent has the address (-1: none given)
  };
  struct BdfMask {
    uint32_t addr;
    std::vector<uint32_t> bits;
    int fallback;
  };
  std::vector<BdfLimit> bdf_limit;                                         // PCI address -> bytes
  std::vector<BdfMask> bdf_mask;                                           // PCI address -> CU bits
  std::atomic<int> unmatched{-1};  // address entries no agent had (-1: not resolved yet)
  State() {
    for (int i = 0; i < kMaxDev; ++i) limit[i] = -1, used[i] = 0;
  }
};

State& st() {
  static State* s = new State();  // never destroyed: frees may arrive from other libraries' destructors
  return *s;
}

// the loaded object whose path contains `stem`, re-opened without loading anything new
void* loaded_library(const char* stem) {
  struct Q {
    const char* stem;
    void* h;
  } q{stem, nullptr};
  dl_iterate_phdr(
      [](struct dl_phdr_info* info, size_t, void* data) -> int {
        Q* q = static_cast<Q*>(data);
        if (info->dlpi_name && std::strstr(info->dlpi_name, q->stem)) {
          q->h = dlopen(info->dlpi_name, RTLD_NOW | RTLD_NOLOAD);
          return q->h != nullptr;
        }
        return 0;
      },
      &q);
  return q.h;
}

template <typename Fn>
Fn real(const char* name, const char* stem) {
  void* p = dlsym(RTLD_NEXT, name);
  if (!p) {
    void* h = loaded_library(stem);
    if (h) p = dlsym(h, name);
  }
  if (!p) {
    std::fprintf(stderr, "gtk-vgpu: cannot resolve %s in %s\n", name, stem);
    std::abort();
  }
  return reinterpret_cast<Fn>(p);
}

// the same, or nullptr while the library is not loaded yet (entry points the guard calls on its own
// initiative, which may run before the program has loaded the runtime)
template <typename Fn>
Fn real_opt(const char* name, const char* stem) {
  void* p = dlsym(RTLD_NEXT, name);
  if (!p) {
    void* h = loaded_library(stem);
    if (h) p = dlsym(h, name);
  }
  return reinterpret_cast<Fn>(p);
}

// resolved once per entry point; a function-local static is initialised thread-safely
#define REAL_HIP(name, type) static const type real_fn = real<type>(#name, "libamdhip64");
#define REAL_HSA(name) static const auto real_fn = real<decltype(&::name)>(#name, "libhsa-runtime64");

// "<cu>[-<cu>][,...]" -> bit words
std::vector<uint32_t> parse_cus(const char* c) {
  std::vector<uint32_t> bits;
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
    for (long cu = a; cu <= b && cu >= 0 && cu < 4096; ++cu) {
      if ((long)bits.size() * 32 <= cu) bits.resize(cu / 32 + 1, 0u);
      bits[cu / 32] |= 1u << (cu % 32);
    }
    if (*c == ',') ++c;
  }
  return bits;
}

// "dddd:bb:dd.f" (hex; the domain may be omitted) -> domain << 16 | bus << 8 | device << 3 | function
bool parse_bdf(const char* t, uint32_t* key) {
  unsigned d = 0, b = 0, v = 0, f = 0;
  if (std::sscanf(t, "%x:%x:%x.%x", &d, &b, &v, &f) != 4) {
    d = 0;
    if (std::sscanf(t, "%x:%x.%x", &b, &v, &f) != 3) return false;
  }
  *key = (d & 0xffffu) << 16 | (b & 0xffu) << 8 | (v & 0x1fu) << 3 | (f & 7u);
  return true;
}

// HSA_CU_MASK syntax: "<ordinal>:<cu>[-<cu>][,...]" parts separated by ';'
std::vector<std::vector<uint32_t>> parse_mask(const std::string& v) {
  std::vector<std::vector<uint32_t>> out;
  size_t i = 0;
  while (i < v.size()) {
    size_t end = v.find(';', i);
    if (end == std::string::npos) end = v.size();
    std::string part = v.substr(i, end - i);
    i = end + 1;
    size_t colon = part.find(':');
    if (colon == std::string::npos) continue;
    int dev = std::atoi(part.c_str());
    if (dev < 0 || dev >= kMaxDev) continue;
    if ((int)out.size() <= dev) out.resize(dev + 1);
    out[dev] = parse_cus(part.c_str() + colon + 1);
  }
  return out;
}

// GPU agents in ROCr's enumeration order (HSA_CU_MASK's ordinals) and each one's global memory pools
// and PCI address.  Built once, on the first queue or allocation, from the real runtime; the
// address-keyed limits and masks of the config are resolved to ordinals then.
struct Agents {
  std::vector<uint64_t> gpus;                       // ordinal -> agent handle
  std::vector<uint32_t> bdf;                        // ordinal -> PCI address key (0xffffffff: unknown)
  std::unordered_map<uint64_t, int> pool_ordinal;   // GPU global pool handle -> ordinal
};

// An address entry no agent has (the runtime reported no BDFID / DOMAIN, or a format mismatch between
// what amdsmi printed and what ROCr reports) must not leave the share silently unenforced:
// it is reported on stderr, counted (gtk_vgpu_unmatched, checked by `gtk doctor --gpu`), and applied to
// the fallback ordinal the plugin wrote next to the address (the device's position among the pod's
// GPUs: right unless the pod renumbers its devices), when there is one.
int unmatched_ordinal(const Agents& a, const char* what, uint32_t addr, int fallback) {
  const bool ok = fallback >= 0 && fallback < (int)a.gpus.size() && fallback < kMaxDev;
  std::fprintf(stderr,
               "gtk-vgpu: %s %04x:%02x:%02x.%x matches none of the %zu GPUs the runtime enumerated%s; %s\n", what,
               addr >> 16, (addr >> 8) & 0xffu, (addr >> 3) & 0x1fu, addr & 7u, a.gpus.size(),
               (!a.bdf.empty() && a.bdf[0] == 0xffffffffu) ? " (the runtime reports no PCI addresses)" : "",
               ok ? "applying it to the fallback ROCr ordinal" : "NO fallback ordinal: this limit is NOT enforced");
  if (ok) std::fprintf(stderr, "gtk-vgpu:   fallback ordinal %d\n", fallback);
  return ok ? fallback : -1;
}

void resolve_bdf_config(const Agents& a) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  auto where = [&](uint32_t addr) -> int {
    for (size_t o = 0; o < a.bdf.size() && o < (size_t)kMaxDev; ++o)
      if (a.bdf[o] == addr) return (int)o;
    return -1;
  };
  int unmatched = 0;
  for (const auto& l : s.bdf_limit) {
    int o = where(l.addr);
    if (o < 0) ++unmatched, o = unmatched_ordinal(a, "hbm_limit_bdf", l.addr, l.fallback);
    if (o >= 0) s.limit[o] = l.bytes;
  }
  for (const auto& m : s.bdf_mask) {
    int o = where(m.addr);
    if (o < 0) ++unmatched, o = unmatched_ordinal(a, "cu_mask_bdf", m.addr, m.fallback);
    if (o >= 0) {
      if ((int)s.mask_bits.size() <= o) s.mask_bits.resize(o + 1);
      s.mask_bits[o] = m.bits;
    }
  }
  s.unmatched = unmatched;
}

// Built once the runtime can enumerate (after hsa_init): a call that comes earlier (an exported
// introspection entry point, a HIP call that does not initialise ROCr) gets an empty table and the next
// call tries again, so the address-keyed config is never resolved against an empty enumeration.
// Readers get an immutable table published with release/acquire.
const Agents& agents() {
  static std::atomic<const Agents*> ready{nullptr};
  static const Agents* const empty = new Agents();
  if (const Agents* p = ready.load(std::memory_order_acquire)) return *p;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (const Agents* p = ready.load(std::memory_order_acquire)) return *p;
  const auto iterate = real_opt<decltype(&::hsa_iterate_agents)>("hsa_iterate_agents", "libhsa-runtime64");
  if (!iterate) return *empty;  // the runtime is not even loaded yet
  Agents* a = new Agents();
  {
    const hsa_status_t e = iterate(
        [](hsa_agent_t ag, void* data) -> hsa_status_t {
          static const auto info = real<decltype(&::hsa_agent_get_info)>("hsa_agent_get_info", "libhsa-runtime64");
          static const auto pools =
              real<decltype(&::hsa_amd_agent_iterate_memory_pools)>("hsa_amd_agent_iterate_memory_pools", "libhsa-runtime64");
          Agents* a = static_cast<Agents*>(data);
          hsa_device_type_t type{};
          if (info(ag, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS || type != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
          a->gpus.push_back(ag.handle);
          uint32_t id = 0, dom = 0;
          const bool known = info(ag, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &id) == HSA_STATUS_SUCCESS &&
                             info(ag, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS;
          a->bdf.push_back(known ? ((dom & 0xffffu) << 16 | (id & 0xffffu)) : 0xffffffffu);
          struct Ctx {
            Agents* a;
            int ordinal;
          } ctx{a, (int)a->gpus.size() - 1};
          pools(
              ag,
              [](hsa_amd_memory_pool_t pool, void* d) -> hsa_status_t {
                static const auto pinfo =
                    real<decltype(&::hsa_amd_memory_pool_get_info)>("hsa_amd_memory_pool_get_info", "libhsa-runtime64");
                Ctx* c = static_cast<Ctx*>(d);
                hsa_amd_segment_t seg{};
                if (pinfo(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) == HSA_STATUS_SUCCESS && seg == HSA_AMD_SEGMENT_GLOBAL)
                  c->a->pool_ordinal[pool.handle] = c->ordinal;
                return HSA_STATUS_SUCCESS;
              },
              &ctx);
          return HSA_STATUS_SUCCESS;
        },
        a);
    if (e != HSA_STATUS_SUCCESS || a->gpus.empty()) {  // not initialised yet (or no GPU): try again later
      delete a;
      return *empty;
    }
  }
  resolve_bdf_config(*a);
  ready.store(a, std::memory_order_release);
  return *a;
}

// ROCr ordinal of HIP device `hip` (HIP may renumber: $HIP_VISIBLE_DEVICES), by PCI address; the HIP
// number itself when the address is unknown
int hip_ordinal(int hip) {
  typedef hipError_t (*F)(char*, int, int);
  static std::atomic<F> cached{nullptr};
  F bus_id = cached.load(std::memory_order_acquire);
  if (!bus_id && (bus_id = real_opt<F>("hipDeviceGetPCIBusId", "libamdhip64")) != nullptr)
    cached.store(bus_id, std::memory_order_release);
  const Agents& a = agents();
  if (!bus_id) return hip;  // no HIP runtime loaded yet
  char bus[64] = {0};
  uint32_t key = 0;
  if (bus_id(bus, (int)sizeof bus, hip) == kSuccess && parse_bdf(bus, &key))
    for (size_t o = 0; o < a.bdf.size(); ++o)
      if (a.bdf[o] == key) return (int)o;
  return hip;
}

int current_ordinal() {
  typedef hipError_t (*G)(int*);
  static const G get_device = real<G>("hipGetDevice", "libamdhip64");
  int dev = 0;
  if (get_device(&dev) != kSuccess) return -1;
  return hip_ordinal(dev);
}

int pool_ordinal(hsa_amd_memory_pool_t pool) {
  const Agents& a = agents();
  auto it = a.pool_ordinal.find(pool.handle);
  return it == a.pool_ordinal.end() ? -1 : it->second;
}

int agent_ordinal(hsa_agent_t agent) {
  const Agents& a = agents();
  for (size_t i = 0; i < a.gpus.size(); ++i)
    if (a.gpus[i] == agent.handle) return (int)i;
  return -1;
}

off_t slot_offset(int i) { return (off_t)(offsetof(Table, slot) + (size_t)i * sizeof(Slot)); }

// another process holds slot i (its fcntl lock); our own lock never shows up in F_GETLK
bool slot_alive(int fd, int i) {
  struct flock fl{};
  fl.l_type = F_WRLCK;
  fl.l_whence = SEEK_SET;
  fl.l_start = slot_offset(i);
  fl.l_len = 1;
  if (fcntl(fd, F_GETLK, &fl) != 0) return true;  // unknown: count it
  return fl.l_type != F_UNLCK;
}

// call with s.mu and the file's flock held: make sure this process owns a slot of the table
bool own_slot(State& s) {
  if (s.mine >= 0 && s.mine_pid == getpid()) return true;
  for (int i = 0; i < kSlots; ++i) {
    if (slot_alive(s.acct_fd, i)) continue;  // another live process's
    struct flock fl{};
    fl.l_type = F_WRLCK;
    fl.l_whence = SEEK_SET;
    fl.l_start = slot_offset(i);
    fl.l_len = 1;
    if (fcntl(s.acct_fd, F_SETLK, &fl) != 0) continue;
    Slot& sl = s.table->slot[i];
    sl.pid = (int32_t)getpid();
    for (int d = 0; d < kMaxDev; ++d) sl.used[d] = 0;  // a dead owner's bytes died with it
    s.mine = i;
    s.mine_pid = getpid();
    return true;
  }
  return false;  // table full: this process falls back to its own budget
}

struct FileLock {  // whole-table critical section across the pod's processes
  int fd;
  explicit FileLock(int f) : fd(f) {
    if (fd >= 0) flock(fd, LOCK_EX);
  }
  ~FileLock() {
    if (fd >= 0) flock(fd, LOCK_UN);
  }
};

// reserve `bytes` on `dev`; false if the share would be exceeded (pod-wide with an acct file)
bool reserve(int dev, size_t bytes) {
  State& s = st();
  if (!s.active || dev < 0 || dev >= kMaxDev || s.limit[dev] < 0) return true;
  std::lock_guard<std::mutex> g(s.mu);
  if (s.table) {
    FileLock fl(s.acct_fd);
    if (own_slot(s)) {
      long long total = 0;
      for (int i = 0; i < kSlots; ++i)
        if (i == s.mine || slot_alive(s.acct_fd, i)) total += s.table->slot[i].used[dev];
      if (total + (long long)bytes > s.limit[dev]) return false;
      s.table->slot[s.mine].used[dev] += (long long)bytes;
      s.used[dev] += (long long)bytes;
      return true;
    }
  }
  if (s.used[dev] + (long long)bytes > s.limit[dev]) return false;
  s.used[dev] += (long long)bytes;
  return true;
}

void unreserve(int dev, size_t bytes) {
  State& s = st();
  if (!s.active || dev < 0 || dev >= kMaxDev || s.limit[dev] < 0) return;
  std::lock_guard<std::mutex> g(s.mu);
  if (s.table && s.mine >= 0 && s.mine_pid == getpid()) {
    FileLock fl(s.acct_fd);
    int64_t& u = s.table->slot[s.mine].used[dev];
    u -= (long long)bytes;
    if (u < 0) u = 0;
  }
  s.used[dev] -= (long long)bytes;
  if (s.used[dev] < 0) s.used[dev] = 0;
}

// bytes in use on `dev` by the whole pod (acct file) or this process
long long pod_used(int dev) {
  State& s = st();
  if (!s.table) return s.used[dev];
  FileLock fl(s.acct_fd);
  long long total = 0;
  for (int i = 0; i < kSlots; ++i)
    if ((i == s.mine && s.mine_pid == getpid()) || slot_alive(s.acct_fd, i)) total += s.table->slot[i].used[dev];
  return total;
}

void open_acct(State& s, const char* path) {
  int fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) {
    std::fprintf(stderr, "gtk-vgpu: accounting file %s unavailable; limits hold per process\n", path);
    return;
  }
  {
    FileLock fl(fd);
    struct stat sb{};
    if (fstat(fd, &sb) != 0 || (sb.st_size < (off_t)sizeof(Table) && ftruncate(fd, sizeof(Table)) != 0)) {
      close(fd);
      return;
    }
  }
  void* m = mmap(nullptr, sizeof(Table), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    return;
  }
  Table* t = static_cast<Table*>(m);
  {
    FileLock fl(fd);
    if (t->magic != kMagic) {  // a fresh (or foreign) file: format it
      std::memset(t, 0, sizeof(Table));
      t->magic = kMagic;
      t->nslots = kSlots;
    }
  }
  s.acct_fd = fd;
  s.table = t;
}

// ordinal of the share's device a pointer was allocated on; (-1, 0) if untracked.  Forget `p` BEFORE
// the runtime frees it: once freed, the address can be handed to another thread's allocation, whose
// entry a late erase would destroy.
std::pair<int, size_t> untrack(void* p) {
  State& s = st();
  if (!s.active || !p) return {-1, 0};
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.ptrs.find(p);
  if (it == s.ptrs.end()) return {-1, 0};
  auto v = it->second;
  s.ptrs.erase(it);
  return v;
}

void set_cu_mask_env() {
  State& s = st();
  if (!s.active) return;
  if (!s.bdf_mask.empty())
    unsetenv("HSA_CU_MASK");  // an ordinal-keyed mask may name other devices; queues get the share's
  else if (!s.cu_mask.empty())
    setenv("HSA_CU_MASK", s.cu_mask.c_str(), 1);
}

const char* config_path() {
  // the plugin's mount wins over anything the pod's environment says
  if (access(GTK_VGPU_FIXED_CONF, R_OK) == 0) return GTK_VGPU_FIXED_CONF;
  const char* env = std::getenv("GTK_VGPU_CONFIG");
  return (env && *env) ? env : nullptr;
}

__attribute__((constructor)) void load_config() {
  const char* path = config_path();
  if (!path) return;
  FILE* f = std::fopen(path, "r");
  if (!f) return;  // no share to enforce: pass-through
  State& s = st();
  char line[4096];
  while (std::fgets(line, sizeof line, f)) {
    char key[64] = {0}, val[4000] = {0}, key_s[64] = {0};
    int dev = -1;
    long long bytes = -1;
    uint32_t addr = 0;
    int fb = -1, nf = 0;
    if ((nf = std::sscanf(line, "hbm_limit_bdf %63s %lld %d", key_s, &bytes, &fb)) >= 2) {
      if (parse_bdf(key_s, &addr) && bytes >= 0) s.bdf_limit.push_back({addr, bytes, nf == 3 ? fb : -1});
    } else if ((nf = std::sscanf(line, "cu_mask_bdf %63s %3999s %d", key_s, val, &fb)) >= 2) {
      if (parse_bdf(key_s, &addr)) s.bdf_mask.push_back({addr, parse_cus(val), nf == 3 ? fb : -1});
    } else if (std::sscanf(line, "hbm_limit %d %lld", &dev, &bytes) == 2) {
      if (dev >= 0 && dev < kMaxDev && bytes >= 0) s.limit[dev] = bytes;
    } else if (std::sscanf(line, "%63s %3999s", key, val) == 2 && std::strcmp(key, "cu_mask") == 0) {
      s.cu_mask = val;
      s.mask_bits = parse_mask(s.cu_mask);
    } else if (std::sscanf(line, "%63s %3999s", key, val) == 2 && std::strcmp(key, "acct") == 0) {
      open_acct(s, val);
    }
  }
  std::fclose(f);
  s.active = true;
  // fork: no thread may hold the lock across it, and the child starts with a budget of its own (HSA
  // state, and so device memory, does not survive a fork); with an acct file it claims its own slot
  pthread_atfork([] { st().mu.lock(); }, [] { st().mu.unlock(); },
                 [] {
                   State& c = st();
                   c.mu.unlock();
                   for (int d = 0; d < kMaxDev; ++d) c.used[d] = 0;
                   c.ptrs.clear();
                   c.handles.clear();
                   c.queues.clear();
                   c.managed.clear();
                   c.mine = -1;
                 });
  set_cu_mask_env();  // before ROCr initialises
  setenv("GTK_VGPU_ACTIVE", "1", 1);  // lets the workload report that the guard is in force
}

// the share's CU bits of `ordinal`, intersected with `want` (nullptr = all CUs); empty = no restriction
std::vector<uint32_t> share_mask(int ordinal, const uint32_t* want, uint32_t want_bits) {
  State& s = st();
  if (!s.active || ordinal < 0 || ordinal >= (int)s.mask_bits.size() || s.mask_bits[ordinal].empty()) return {};
  std::vector<uint32_t> m = s.mask_bits[ordinal];
  if (want) {
    bool any = false;
    for (size_t w = 0; w < m.size(); ++w) {
      const uint32_t x = m[w] & (w < want_bits / 32 ? want[w] : 0u);
      any |= x != 0;
      if (any) break;
    }
    if (any)  // an empty intersection would stop the queue: the share's own mask applies instead
      for (size_t w = 0; w < m.size(); ++w) m[w] &= (w < want_bits / 32 ? want[w] : 0u);
  }
  return m;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- ROCr: initialisation and queues

// Every HIP program initialises ROCr through here, whatever its first HIP call: the share's mask is
// put back into the environment ROCr is about to read.
__attribute__((visibility("default"))) hsa_status_t hsa_init() {
  set_cu_mask_env();
  REAL_HSA(hsa_init);
  return real_fn();
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_create(
    hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type, void (*callback)(hsa_status_t, hsa_queue_t*, void*),
    void* data, uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
  REAL_HSA(hsa_queue_create);
  hsa_status_t e = real_fn(agent, size, type, callback, data, private_segment_size, group_segment_size, queue);
  State& s = st();
  if (e != HSA_STATUS_SUCCESS || !queue || !*queue || !s.active || (s.mask_bits.empty() && s.bdf_mask.empty())) return e;
  const int ord = agent_ordinal(agent);  // resolves the address-keyed masks on first use
  std::vector<uint32_t> m = share_mask(ord, nullptr, 0);
  if (m.empty()) return e;
  {
    std::lock_guard<std::mutex> g(s.mu);
    s.queues[*queue] = ord;
  }
  static const auto set_mask = real<decltype(&::hsa_amd_queue_cu_set_mask)>("hsa_amd_queue_cu_set_mask", "libhsa-runtime64");
  const hsa_status_t me = set_mask(*queue, (uint32_t)(m.size() * 32), m.data());
  if (me != HSA_STATUS_SUCCESS && me != HSA_STATUS_INFO_BREAK)
    std::fprintf(stderr, "gtk-vgpu: applying the share's CU mask to a queue failed (%d)\n", (int)me);
  return e;
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_destroy(hsa_queue_t* queue) {
  State& s = st();
  if (s.active && queue) {
    std::lock_guard<std::mutex> g(s.mu);
    s.queues.erase(queue);
  }
  REAL_HSA(hsa_queue_destroy);
  return real_fn(queue);
}

// A program's own CU mask (hipExtStreamCreateWithCUMask) is narrowed to the share.
__attribute__((visibility("default"))) hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* queue,
                                                                               uint32_t num_cu_mask_count,
                                                                               const uint32_t* cu_mask) {
  REAL_HSA(hsa_amd_queue_cu_set_mask);
  State& s = st();
  int ord = -1;
  if (s.active && queue) {
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.queues.find(queue);
    if (it != s.queues.end()) ord = it->second;
  }
  std::vector<uint32_t> m = share_mask(ord, cu_mask, num_cu_mask_count);
  if (m.empty()) return real_fn(queue, num_cu_mask_count, cu_mask);
  return real_fn(queue, (uint32_t)(m.size() * 32), m.data());
}

// ---------------------------------------------------------------- ROCr: device memory

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t pool, size_t size,
                                                                                  uint32_t flags, void** ptr) {
  REAL_HSA(hsa_amd_memory_pool_allocate);
  State& s = st();
  if (!s.active) return real_fn(pool, size, flags, ptr);
  const int dev = pool_ordinal(pool);
  if (!reserve(dev, size)) {
    if (ptr) *ptr = nullptr;
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t e = real_fn(pool, size, flags, ptr);
  if (dev < 0 || dev >= kMaxDev || s.limit[dev] < 0) return e;
  if (e != HSA_STATUS_SUCCESS || !ptr || !*ptr) {
    unreserve(dev, size);
    return e;
  }
  std::lock_guard<std::mutex> g(s.mu);
  s.ptrs[*ptr] = {dev, size};
  return e;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  REAL_HSA(hsa_amd_memory_pool_free);
  auto v = untrack(ptr);
  hsa_status_t e = real_fn(ptr);
  if (v.first >= 0) {
    if (e == HSA_STATUS_SUCCESS) {
      unreserve(v.first, v.second);
    } else {  // the free failed: the allocation is still live
      std::lock_guard<std::mutex> g(st().mu);
      st().ptrs[ptr] = v;
    }
  }
  return e;
}

// physical memory behind the virtual-memory API (hipMemCreate, expandable caching-allocator segments)
__attribute__((visibility("default"))) hsa_status_t hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t pool, size_t size,
                                                                                hsa_amd_memory_type_t type, uint64_t flags,
                                                                                hsa_amd_vmem_alloc_handle_t* handle) {
  REAL_HSA(hsa_amd_vmem_handle_create);
  State& s = st();
  if (!s.active) return real_fn(pool, size, type, flags, handle);
  const int dev = pool_ordinal(pool);
  if (!reserve(dev, size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t e = real_fn(pool, size, type, flags, handle);
  if (dev < 0 || dev >= kMaxDev || s.limit[dev] < 0) return e;
  if (e != HSA_STATUS_SUCCESS || !handle) {
    unreserve(dev, size);
    return e;
  }
  std::lock_guard<std::mutex> g(s.mu);
  s.handles[handle->handle] = {dev, size};
  return e;
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_vmem_handle_release(hsa_amd_vmem_alloc_handle_t handle) {
  REAL_HSA(hsa_amd_vmem_handle_release);
  State& s = st();
  std::pair<int, size_t> v{-1, 0};
  if (s.active) {  // forget the handle before the runtime can reuse its value
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.handles.find(handle.handle);
    if (it != s.handles.end()) {
      v = it->second;
      s.handles.erase(it);
    }
  }
  hsa_status_t e = real_fn(handle);
  if (v.first >= 0) {
    if (e == HSA_STATUS_SUCCESS) {
      unreserve(v.first, v.second);
    } else {
      std::lock_guard<std::mutex> g(s.mu);
      s.handles[handle.handle] = v;
    }
  }
  return e;
}

// ---------------------------------------------------------------- HIP: what the process is told

// the share is the device's size as far as this process can tell
__attribute__((visibility("default"))) hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  typedef hipError_t (*F)(size_t*, size_t*);
  REAL_HIP(hipMemGetInfo, F);
  hipError_t e = real_fn(free_b, total_b);
  State& s = st();
  if (e != kSuccess || !s.active) return e;
  const int dev = current_ordinal();
  if (dev < 0 || dev >= kMaxDev || s.limit[dev] < 0) return e;
  std::lock_guard<std::mutex> g(s.mu);
  const long long left = s.limit[dev] - pod_used(dev);
  if (total_b && (long long)*total_b > s.limit[dev]) *total_b = (size_t)s.limit[dev];
  if (free_b && (long long)*free_b > left) *free_b = (size_t)(left > 0 ? left : 0);
  return e;
}

// Managed memory the runtime did not place in a device pool (HMM: system pages that migrate into HBM
// when a kernel touches them) would bypass the pool hooks: charged here, in full, to the current device.
// The charge follows the real call: a runtime that does take the block from a device pool has charged
// (and checked) it in the pool hook already, and a charge taken beforehand would count it twice while
// that hook decides.  A block over the share is handed back before the caller sees it.
__attribute__((visibility("default"))) hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  typedef hipError_t (*F)(void**, size_t, unsigned int);
  typedef hipError_t (*FreeF)(void*);
  REAL_HIP(hipMallocManaged, F);
  static const FreeF real_free = real<FreeF>("hipFree", "libamdhip64");
  State& s = st();
  if (!s.active) return real_fn(ptr, size, flags);
  const int dev = current_ordinal();
  hipError_t e = real_fn(ptr, size, flags);
  if (e != kSuccess || !ptr || !*ptr) return e;
  {
    std::lock_guard<std::mutex> g(s.mu);
    if (s.ptrs.count(*ptr)) return e;  // the runtime took it from a device pool: counted there
  }
  if (!reserve(dev, size)) {
    real_free(*ptr);
    *ptr = nullptr;
    return 2;  // hipErrorOutOfMemory
  }
  if (dev >= 0 && dev < kMaxDev && s.limit[dev] >= 0) {
    std::lock_guard<std::mutex> g(s.mu);
    s.managed[*ptr] = {dev, size};
  }
  return e;
}

__attribute__((visibility("default"))) hipError_t hipFree(void* ptr) {
  typedef hipError_t (*F)(void*);
  REAL_HIP(hipFree, F);
  State& s = st();
  std::pair<int, size_t> v{-1, 0};
  if (s.active && ptr) {  // forget it before the address can be handed out again
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.managed.find(ptr);
    if (it != s.managed.end()) {
      v = it->second;
      s.managed.erase(it);
    }
  }
  hipError_t e = real_fn(ptr);
  if (v.first >= 0) {
    if (e == kSuccess) {
      unreserve(v.first, v.second);
    } else {
      std::lock_guard<std::mutex> g(s.mu);
      s.managed[ptr] = v;
    }
  }
  return e;
}

// ROCr ordinal the HIP device `hip` maps to (tests: the address-keyed config under renumbering)
__attribute__((visibility("default"))) int gtk_vgpu_hip_ordinal(int hip) { return hip_ordinal(hip); }

// introspection for tests and the workload's report: bytes in use / limit on `dev` (-1: no limit)
__attribute__((visibility("default"))) long long gtk_vgpu_used(int dev) {
  if (dev < 0 || dev >= kMaxDev) return -1;
  std::lock_guard<std::mutex> g(st().mu);
  return st().used[dev];
}

// bytes in use on `dev` by every live process sharing the accounting file (= gtk_vgpu_used without one)
__attribute__((visibility("default"))) long long gtk_vgpu_pod_used(int dev) {
  if (dev < 0 || dev >= kMaxDev) return -1;
  std::lock_guard<std::mutex> g(st().mu);
  return pod_used(dev);
}

__attribute__((visibility("default"))) long long gtk_vgpu_limit(int dev) {
  if (dev < 0 || dev >= kMaxDev) return -1;
  std::lock_guard<std::mutex> g(st().mu);
  return st().limit[dev];
}

// address-keyed config entries no GPU agent had (each reported on stderr; applied to its fallback
// ordinal when the config names one); -1 while the runtime has not enumerated its agents yet
__attribute__((visibility("default"))) int gtk_vgpu_unmatched() {
  agents();  // resolves the config once the runtime can enumerate
  return st().unmatched.load();
}

// queues of this process the share's mask was applied to
__attribute__((visibility("default"))) int gtk_vgpu_masked_queues() {
  std::lock_guard<std::mutex> g(st().mu);
  return (int)st().queues.size();
}

}  // extern "C"
