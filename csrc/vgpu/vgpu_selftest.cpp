// Host-only stress test of the vGPU guard (csrc/vgpu/vgpu_guard.cpp) under ThreadSanitizer and
// AddressSanitizer/UBSan: the guard's sources are linked into this binary, the
// stand-in HIP runtime (fake_hip.cpp) is its "libamdhip64", and many threads allocate and free
// concurrently against one budget (device-pool allocations and HIP-level managed ones).  The test
// process sets GTK_VGPU_CONFIG before start (the guard's constructor reads it before main); the config
// may name the device by ordinal or by PCI address (resolved when the runtime first enumerates).
// Checks: no allocation ever succeeds past the limit, every byte is returned, hipMemGetInfo stays
// consistent, and (with an ``acct`` file) forked children share the parent's budget.
//
//     GTK_VGPU_CONFIG=cfg ./vgpu_selftest_tsan [threads] [iters]
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

extern "C" {
int hipMalloc(void** p, size_t n);
int hipFree(void* p);
int hipMallocAsync(void** p, size_t n, void* stream);
int hipMallocManaged(void** p, size_t n, unsigned int flags);
int hipFreeAsync(void* p, void* stream);
int hipMemGetInfo(size_t* f, size_t* t);
long long gtk_vgpu_used(int dev);
long long gtk_vgpu_limit(int dev);
long long gtk_vgpu_pod_used(int dev);
}

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 16;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  size_t f0 = 0, t0 = 0;
  hipMemGetInfo(&f0, &t0);  // first runtime call: an address-keyed limit is resolved here
  const long long limit = gtk_vgpu_limit(0);
  if (limit <= 0) return fail("no hbm_limit for ordinal 0 in GTK_VGPU_CONFIG");
  std::atomic<long long> live{0}, peak{0}, ooms{0}, oks{0};
  std::atomic<int> over{0}, bad_free{0}, bad_oom{0};
  std::vector<std::thread> ts;
  std::atomic<int> started{0};
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&, t] {
      started++;
      while (started.load() < threads) std::this_thread::yield();  // all threads contend from the start
      std::mt19937_64 rng(1234 + t);
      struct Held {
        void* p;
        size_t n;
        bool managed;
      };
      std::vector<Held> held;
      for (int i = 0; i < iters; ++i) {
        if (!held.empty() && (rng() % 3 == 0 || held.size() > 16)) {
          const Held h = held.back();
          held.pop_back();
          live -= (long long)h.n;
          if ((h.managed || (rng() & 1)) ? hipFree(h.p) : hipFreeAsync(h.p, nullptr)) bad_free++;
          continue;
        }
        const size_t n = (size_t)(1 + rng() % (limit / 4));
        void* p = nullptr;
        // reserve in the shadow count first: `live` only ever overstates what the guard holds
        const long long now = (live += (long long)n);
        const int kind = (int)(rng() % 3);  // pool, stream-ordered pool, managed (charged at the HIP level)
        const int e = kind == 0 ? hipMalloc(&p, n) : kind == 1 ? hipMallocAsync(&p, n, nullptr) : hipMallocManaged(&p, n, 1);
        if (e == 0) {
          oks++;
          held.push_back({p, n, kind == 2});
          long long pk = peak.load();
          while (now > pk && !peak.compare_exchange_weak(pk, now)) {
          }
          if (gtk_vgpu_used(0) > limit) over++;
        } else {
          live -= (long long)n;
          if (e != 2 || p != nullptr) {  // must be hipErrorOutOfMemory with a null pointer
            if (bad_oom++ == 0) std::fprintf(stderr, "refusal: e=%d p=%p n=%zu\n", e, p, n);
          }
          ooms++;
        }
      }
      for (const Held& h : held) {
        live -= (long long)h.n;
        hipFree(h.p);
      }
    });
  }
  for (auto& t : ts) t.join();
  if (over.load()) return fail("an allocation passed the limit");
  if (bad_free.load()) return fail("a free of a live allocation failed");
  if (bad_oom.load()) return fail("a refusal was not hipErrorOutOfMemory with a null pointer");
  if (gtk_vgpu_used(0) != 0) return fail("bytes leaked in the guard's accounting");
  if (ooms.load() == 0) return fail("the stress never reached the limit (test too small)");
  size_t f = 0, tot = 0;
  hipMemGetInfo(&f, &tot);
  if ((long long)tot != limit || (long long)f != limit) return fail("hipMemGetInfo does not report the share");
  // forked children draw from the same pod budget when an acct file is configured
  if (getenv("SELFTEST_ACCT")) {
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)(limit * 3 / 4))) return fail("parent could not take 3/4 of the share");
    pid_t c = fork();
    if (c == 0) {
      void* q = nullptr;
      const int e = hipMalloc(&q, (size_t)(limit / 2));  // 3/4 + 1/2 > 1: refused for the pod
      const int e2 = hipMalloc(&q, (size_t)(limit / 8));
      _exit(e == 2 && e2 == 0 && gtk_vgpu_pod_used(0) == limit * 3 / 4 + limit / 8 ? 0 : 3);
    }
    int status = 0;
    waitpid(c, &status, 0);
    if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) return fail("forked child did not share the pod budget");
    if (gtk_vgpu_pod_used(0) != limit * 3 / 4) return fail("the dead child's bytes were not released");
    hipFree(p);
  }
  std::printf("{\"threads\": %d, \"iters\": %d, \"ok\": %lld, \"oom\": %lld, \"peak_shadow\": %lld, \"limit\": %lld}\n", threads,
              iters, oks.load(), ooms.load(), peak.load(), limit);
  return 0;
}
