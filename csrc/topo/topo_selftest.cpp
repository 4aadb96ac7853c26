// Host-only sanitizer build of the KFD sysfs reader (CPU-side C++ under
// -fsanitize=address,undefined).  The reader parses files the node's kernel writes; a driver bug, a
// partial hot-unplug or a half-written RAS file can leave them in any state, and the device plugin must
// survive it.  tests/test_topo_reader_asan.py writes corrupted copies of the 8 x MI355X fixture tree and
// runs this binary over them: each tree must give a result or a clean exception, never a sanitizer
// report.
//
//   topo_selftest <kfd root> <drm root> <pci root> <numa root> <ib root> [five more roots ...]
//
// One line per tree: "ok <gpus> <nics>" or "raised <message>".
#define GTK_TOPO_NO_PYTHON 1
#include "topo_reader.cpp"

#include <cstdio>

int main(int argc, char** argv) {
  if (argc < 6 || (argc - 1) % 5 != 0) {
    std::fprintf(stderr, "usage: %s <kfd> <drm> <pci> <node> <ib> [...]\n", argv[0]);
    return 2;
  }
  for (int i = 1; i + 4 < argc; i += 5) {
    try {
      Result r = discover_sysfs_impl(argv[i], argv[i + 1]);
      read_host_affinity(r, argv[i + 2], argv[i + 3]);
      read_nics(r, argv[i + 2], argv[i + 4]);
      const size_t n = r.devs.size();
      for (const auto* m : {&r.link_type, &r.hops, &r.p2p})
        if (m->size() != n) throw std::logic_error("matrix size mismatch");
      std::printf("ok %zu %zu\n", n, r.nics.size());
    } catch (const std::exception& e) {
      std::string msg = e.what();
      for (auto& c : msg)
        if (c == '\n') c = ' ';
      std::printf("raised %.200s\n", msg.c_str());
    }
  }
  return 0;
}
