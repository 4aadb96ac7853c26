// libgtk_vgpu.so — the container-side tier of a time-sliced GPU share (Gaia's two-tier vGPU).
//
// Reference: the Gaia paper (p.3 §III.A "GPU resource virtualization") splits a GPU into vGPUs in
// its device plugin and enforces each vGPU's limits inside the container by intercepting the GPU API
// (GaiaGPU's interception library).  On MI355X the device plugin already gives a pod holding part of
// a GPU its slices' compute units (HSA_CU_MASK, topology/shares.py) and its HBM share
// (GTK_GPU_FRACTION); both were cooperative: a container could rewrite its environment, and only the
// framework's own training entry point capped its allocator.  This library, which Allocate mounts
// into the container and preloads (deviceplugin/plugin.py, --share-guard), makes them hold for any
// HIP program in the pod:
//
//   * HBM: every device allocation of the process (hipMalloc, hipExtMallocWithFlags, hipMallocManaged,
//     hipMallocPitch, hipMallocAsync, hipMallocFromPoolAsync, hipMemCreate) is counted against the
//     device's limit and refused with hipErrorOutOfMemory beyond it; frees give it back; hipMemGetInfo
//     reports the share as the device's total, so caching allocators size themselves to it.
//   * CUs: HSA_CU_MASK is set from the mounted config before the program's own code runs (a
//     constructor of a preloaded library runs before main and before any HIP call, and the ROCr
//     runtime reads the variable when it initialises), whatever the container's environment says;
//     and set again at the first intercepted HIP call (the calls a program makes first: hipInit,
//     hipGetDeviceCount, hipSetDevice, hipGetDevice, the allocators), in case the program itself
//     rewrote it before initialising the runtime.
//
// The config is the read-only file ``$GTK_VGPU_CONFIG`` (default /etc/gtk-vgpu.conf) the plugin
// writes per allocation:
//     hbm_limit <HIP ordinal> <bytes>
//     cu_mask <HSA_CU_MASK value>
//     acct <path>                  (optional) pod-wide accounting file, shared read-write
// No file: the library is inert (pure pass-through).  Without ``acct`` the limit holds per process.
// With it, every process of the pod that maps the file draws from one budget: the file is a table of
// per-process slots (bytes in use per device); a process owns its slot by holding an fcntl write lock
// on the slot's first byte, so the kernel drops a crashed process's usage with its lock — whatever PID
// namespace the pod's containers live in — and the next process reuses the slot.
//
// The real HIP entry points are found with dlsym(RTLD_NEXT); when the runtime was loaded RTLD_LOCAL
// (the PyTorch wheel's bundled libamdhip64, brought in by Python's extension loader) RTLD_NEXT does
// not see it, so the loaded objects are searched for libamdhip64 and it is re-opened RTLD_NOLOAD.
// Host-only C++ (g++): no device code, no HIP headers (the few types needed are ABI-identical
// stand-ins), no link against any HIP library.
#include <dlfcn.h>
#include <fcntl.h>
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

namespace {

typedef int hipError_t;  // enum hipError_t: int-sized
constexpr hipError_t kSuccess = 0;
constexpr hipError_t kOutOfMemory = 2;  // hipErrorOutOfMemory
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
  long long limit[kMaxDev];  // bytes; < 0 = no limit on that ordinal
  long long used[kMaxDev];
  std::unordered_map<void*, std::pair<int, size_t>> ptrs;
  std::unordered_map<unsigned long long, std::pair<int, size_t>> handles;  // hipMemCreate handles
  std::string cu_mask;
  State() {
    for (int i = 0; i < kMaxDev; ++i) limit[i] = -1, used[i] = 0;
  }
};

State& st() {
  static State* s = new State();  // never destroyed: frees may arrive from other libraries' destructors
  return *s;
}

void* hip_runtime_handle() {
  static void* h = nullptr;
  static std::once_flag once;
  std::call_once(once, [] {
    dl_iterate_phdr(
        [](struct dl_phdr_info* info, size_t, void*) -> int {
          if (info->dlpi_name && std::strstr(info->dlpi_name, "libamdhip64")) {
            h = dlopen(info->dlpi_name, RTLD_NOW | RTLD_NOLOAD);
            return h != nullptr;
          }
          return 0;
        },
        nullptr);
  });
  return h;
}

template <typename Fn>
Fn real(const char* name) {
  void* p = dlsym(RTLD_NEXT, name);
  if (!p) {
    void* h = hip_runtime_handle();
    if (h) p = dlsym(h, name);
  }
  if (!p) {
    std::fprintf(stderr, "gtk-vgpu: cannot resolve %s in the HIP runtime\n", name);
    std::abort();
  }
  return reinterpret_cast<Fn>(p);
}

// resolved once per entry point; a function-local static is initialised thread-safely
#define REAL(name, type) static const type real_fn = real<type>(#name);

// The runtime reads HSA_CU_MASK once, when the process's first HIP call initialises it.  A program may
// have rewritten the variable after the constructor below set it (Python's os.environ before
// `import torch`), so every intercepted entry point sets it back once, before its first call into the
// runtime: if that call is the one that initialises it, the runtime reads the share's mask.
std::atomic<bool> g_mask_reasserted{false};

void reassert_cu_mask();

int current_device() {
  typedef hipError_t (*F)(int*);
  REAL(hipGetDevice, F);
  int d = 0;
  if (real_fn(&d) != kSuccess || d < 0 || d >= kMaxDev) return 0;
  return d;
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

void track(void* p, int dev, size_t bytes) {
  State& s = st();
  if (!s.active || !p) return;
  std::lock_guard<std::mutex> g(s.mu);
  s.ptrs[p] = {dev, bytes};
}

// forget `p` BEFORE the runtime frees it: once freed, the address can be handed to another thread's
// allocation, whose entry a late erase would destroy.  -> (device, bytes), or (-1, 0) if untracked
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

// the free went through: give the bytes back; it failed: the allocation is still live
void settle_free(void* p, std::pair<int, size_t> v, hipError_t e) {
  if (v.first < 0) return;
  if (e == kSuccess) {
    unreserve(v.first, v.second);
  } else {
    track(p, v.first, v.second);
  }
}

// one allocation through `call` (which performs the real allocation into *ptr)
template <typename Call>
hipError_t guarded(void** ptr, size_t bytes, Call call) {
  const int dev = current_device();
  if (!reserve(dev, bytes)) {
    if (ptr) *ptr = nullptr;
    return kOutOfMemory;
  }
  hipError_t e = call();
  if (e != kSuccess || !ptr || !*ptr) {
    unreserve(dev, bytes);
    return e;
  }
  track(*ptr, dev, bytes);
  return e;
}

__attribute__((constructor)) void load_config() {
  const char* path = std::getenv("GTK_VGPU_CONFIG");
  if (!path || !*path) path = "/etc/gtk-vgpu.conf";
  FILE* f = std::fopen(path, "r");
  if (!f) return;  // no share to enforce: pass-through
  State& s = st();
  char line[4096];
  while (std::fgets(line, sizeof line, f)) {
    char key[64] = {0}, val[4000] = {0};
    int dev = -1;
    long long bytes = -1;
    if (std::sscanf(line, "hbm_limit %d %lld", &dev, &bytes) == 2) {
      if (dev >= 0 && dev < kMaxDev && bytes >= 0) s.limit[dev] = bytes;
    } else if (std::sscanf(line, "%63s %3999s", key, val) == 2 && std::strcmp(key, "cu_mask") == 0) {
      s.cu_mask = val;
    } else if (std::sscanf(line, "%63s %3999s", key, val) == 2 && std::strcmp(key, "acct") == 0) {
      open_acct(s, val);
    }
  }
  std::fclose(f);
  s.active = true;
  // fork: no thread may hold the lock across it, and the child starts with a budget of its own (HIP
  // state, and so device memory, does not survive a fork); with an acct file it claims its own slot
  pthread_atfork([] { st().mu.lock(); }, [] { st().mu.unlock(); },
                 [] {
                   State& c = st();
                   c.mu.unlock();
                   for (int d = 0; d < kMaxDev; ++d) c.used[d] = 0;
                   c.ptrs.clear();
                   c.handles.clear();
                   c.mine = -1;
                 });
  if (!s.cu_mask.empty()) setenv("HSA_CU_MASK", s.cu_mask.c_str(), 1);  // before ROCr initialises
  setenv("GTK_VGPU_ACTIVE", "1", 1);  // lets the workload report that the guard is in force
}

void reassert_cu_mask() {
  if (g_mask_reasserted.load(std::memory_order_acquire)) return;
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  if (g_mask_reasserted.load(std::memory_order_relaxed)) return;
  if (s.active && !s.cu_mask.empty()) setenv("HSA_CU_MASK", s.cu_mask.c_str(), 1);
  g_mask_reasserted.store(true, std::memory_order_release);
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) hipError_t hipMalloc(void** ptr, size_t size) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t);
  REAL(hipMalloc, F);
  return guarded(ptr, size, [&] { return real_fn(ptr, size); });
}

__attribute__((visibility("default"))) hipError_t hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t, unsigned int);
  REAL(hipExtMallocWithFlags, F);
  return guarded(ptr, size, [&] { return real_fn(ptr, size, flags); });
}

__attribute__((visibility("default"))) hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t, unsigned int);
  REAL(hipMallocManaged, F);
  return guarded(ptr, size, [&] { return real_fn(ptr, size, flags); });
}

__attribute__((visibility("default"))) hipError_t hipMallocAsync(void** ptr, size_t size, void* stream) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t, void*);
  REAL(hipMallocAsync, F);
  return guarded(ptr, size, [&] { return real_fn(ptr, size, stream); });
}

__attribute__((visibility("default"))) hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, void* pool, void* stream) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t, void*, void*);
  REAL(hipMallocFromPoolAsync, F);
  return guarded(ptr, size, [&] { return real_fn(ptr, size, pool, stream); });
}

__attribute__((visibility("default"))) hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t*, size_t, size_t);
  REAL(hipMallocPitch, F);
  // the pitch is not known before the call: reserve the unpadded size, then settle to pitch*height
  const int dev = current_device();
  const size_t want = width * height;
  if (!reserve(dev, want)) {
    if (ptr) *ptr = nullptr;
    return kOutOfMemory;
  }
  hipError_t e = real_fn(ptr, pitch, width, height);
  if (e != kSuccess || !ptr || !*ptr) {
    unreserve(dev, want);
    return e;
  }
  const size_t got = (pitch ? *pitch : width) * height;
  if (got > want && !reserve(dev, got - want)) {
    typedef hipError_t (*G)(void*);
    REAL(hipFree, G);
    real_fn(*ptr);
    *ptr = nullptr;
    unreserve(dev, want);
    return kOutOfMemory;
  }
  track(*ptr, dev, got > want ? got : want);
  return e;
}

__attribute__((visibility("default"))) hipError_t hipFree(void* ptr) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void*);
  REAL(hipFree, F);
  auto v = untrack(ptr);
  hipError_t e = real_fn(ptr);
  settle_free(ptr, v, e);
  return e;
}

__attribute__((visibility("default"))) hipError_t hipFreeAsync(void* ptr, void* stream) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void*, void*);
  REAL(hipFreeAsync, F);
  auto v = untrack(ptr);
  hipError_t e = real_fn(ptr, stream);
  settle_free(ptr, v, e);
  return e;
}

// hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size, const hipMemAllocationProp* prop,
// unsigned long long flags): the handle is an opaque pointer-sized value
__attribute__((visibility("default"))) hipError_t hipMemCreate(void** handle, size_t size, const void* prop,
                                                                unsigned long long flags) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void**, size_t, const void*, unsigned long long);
  REAL(hipMemCreate, F);
  const int dev = current_device();
  if (!reserve(dev, size)) return kOutOfMemory;
  hipError_t e = real_fn(handle, size, prop, flags);
  if (e != kSuccess || !handle) {
    unreserve(dev, size);
    return e;
  }
  State& s = st();
  if (s.active) {
    std::lock_guard<std::mutex> g(s.mu);
    s.handles[(unsigned long long)(*handle)] = {dev, size};
  }
  return e;
}

__attribute__((visibility("default"))) hipError_t hipMemRelease(void* handle) {
  reassert_cu_mask();
  typedef hipError_t (*F)(void*);
  REAL(hipMemRelease, F);
  State& s = st();
  int dev = -1;
  size_t bytes = 0;
  if (s.active) {  // forget the handle before the runtime can reuse its value
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.handles.find((unsigned long long)handle);
    if (it != s.handles.end()) {
      dev = it->second.first;
      bytes = it->second.second;
      s.handles.erase(it);
    }
  }
  hipError_t e = real_fn(handle);
  if (dev >= 0) {
    if (e == kSuccess) {
      unreserve(dev, bytes);
    } else {
      std::lock_guard<std::mutex> g(s.mu);
      s.handles[(unsigned long long)handle] = {dev, bytes};
    }
  }
  return e;
}

// the share is the device's size as far as this process can tell
__attribute__((visibility("default"))) hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  reassert_cu_mask();
  typedef hipError_t (*F)(size_t*, size_t*);
  REAL(hipMemGetInfo, F);
  hipError_t e = real_fn(free_b, total_b);
  State& s = st();
  const int dev = current_device();
  if (e != kSuccess || !s.active || s.limit[dev] < 0) return e;
  std::lock_guard<std::mutex> g(s.mu);
  const long long left = s.limit[dev] - pod_used(dev);
  if (total_b && (long long)*total_b > s.limit[dev]) *total_b = (size_t)s.limit[dev];
  if (free_b && (long long)*free_b > left) *free_b = (size_t)(left > 0 ? left : 0);
  return e;
}

// The calls a program usually makes first (torch: hipGetDeviceCount), which initialise the runtime:
// pass-through after the mask is set back.
__attribute__((visibility("default"))) hipError_t hipInit(unsigned int flags) {
  reassert_cu_mask();
  typedef hipError_t (*F)(unsigned int);
  REAL(hipInit, F);
  return real_fn(flags);
}

__attribute__((visibility("default"))) hipError_t hipGetDeviceCount(int* count) {
  reassert_cu_mask();
  typedef hipError_t (*F)(int*);
  REAL(hipGetDeviceCount, F);
  return real_fn(count);
}

__attribute__((visibility("default"))) hipError_t hipSetDevice(int dev) {
  reassert_cu_mask();
  typedef hipError_t (*F)(int);
  REAL(hipSetDevice, F);
  return real_fn(dev);
}

__attribute__((visibility("default"))) hipError_t hipGetDevice(int* dev) {
  reassert_cu_mask();
  typedef hipError_t (*F)(int*);
  REAL(hipGetDevice, F);
  return real_fn(dev);
}

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
  return (dev >= 0 && dev < kMaxDev) ? st().limit[dev] : -1;
}

}  // extern "C"
