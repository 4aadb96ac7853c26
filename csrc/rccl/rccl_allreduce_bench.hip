// Standalone placement validator (no Python): run inside the pod on its allocated GPUs.
//
//   rccl_allreduce_bench [--devices 0,1,2,3] [--min 8] [--max 16G] [--factor 2] [--dtype bf16]
//                        [--iters 20] [--warmup 5] [--inplace] [--no-check] [--json]
//
// Default device list: every visible device (the container only sees its GROUP, design.md:239,
// via /dev/dri/renderD* mounts).  Prints an nccl-tests-style table or JSON lines.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "rccl_core.h"

using namespace gtk;

static size_t parse_size(const std::string& s) {
  char* end = nullptr;
  double v = strtod(s.c_str(), &end);
  std::string suf = end ? std::string(end) : "";
  double mul = 1;
  if (suf == "K" || suf == "k") mul = 1024.0;
  else if (suf == "M" || suf == "m") mul = 1024.0 * 1024;
  else if (suf == "G" || suf == "g") mul = 1024.0 * 1024 * 1024;
  return (size_t)(v * mul);
}

int main(int argc, char** argv) {
  std::vector<int> devs;
  size_t mn = 8, mx = (size_t)1 << 30;
  int factor = 2, iters = 20, warmup = 5;
  std::string dtype = "bf16";
  bool inplace = false, check = true, json = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--devices") {
      std::string s = next();
      size_t p = 0;
      while (p < s.size()) {
        size_t q = s.find(',', p);
        devs.push_back(std::stoi(s.substr(p, q == std::string::npos ? std::string::npos : q - p)));
        if (q == std::string::npos) break;
        p = q + 1;
      }
    } else if (a == "--min") mn = parse_size(next());
    else if (a == "--max") mx = parse_size(next());
    else if (a == "--factor") factor = std::stoi(next());
    else if (a == "--dtype") dtype = next();
    else if (a == "--iters") iters = std::stoi(next());
    else if (a == "--warmup") warmup = std::stoi(next());
    else if (a == "--inplace") inplace = true;
    else if (a == "--no-check") check = false;
    else if (a == "--json") json = true;
    else {
      fprintf(stderr, "usage: %s [--devices a,b,..] [--min B] [--max B] [--factor F] [--dtype bf16|fp16|fp32] "
                      "[--iters N] [--warmup N] [--inplace] [--no-check] [--json]\n", argv[0]);
      return 2;
    }
  }
  try {
    if (devs.empty()) {
      int n = 0;
      RCCL_HIP_CHECK(hipGetDeviceCount(&n));
      for (int i = 0; i < n; ++i) devs.push_back(i);
    }
    LocalGroup g(devs);
    if (!json) {
      printf("# rccl_allreduce_bench: k=%zu dtype=%s %s\n", devs.size(), dtype.c_str(), inplace ? "in-place" : "out-of-place");
      printf("%14s %14s %12s %12s %12s %8s\n", "size(B)", "count", "time(us)", "algbw(GB/s)", "busbw(GB/s)", "wrong");
    }
    double peak_bus = 0, peak_alg = 0;
    unsigned long long wrong_total = 0;
    for (size_t b : size_sweep(mn, mx, factor)) {
      SweepPoint p = g.run(b, dtype, iters, warmup, inplace, check);
      peak_bus = std::max(peak_bus, p.busbw);
      peak_alg = std::max(peak_alg, p.algbw);
      wrong_total += p.wrong;
      if (json)
        printf("{\"bytes\":%zu,\"count\":%zu,\"time_us\":%.3f,\"algbw_gbps\":%.3f,\"busbw_gbps\":%.3f,\"wrong\":%llu}\n",
               p.bytes, p.count, p.time_us, p.algbw, p.busbw, p.wrong);
      else
        printf("%14zu %14zu %12.2f %12.2f %12.2f %8llu\n", p.bytes, p.count, p.time_us, p.algbw, p.busbw, p.wrong);
    }
    if (json)
      printf("{\"summary\":true,\"k\":%zu,\"peak_algbw_gbps\":%.3f,\"peak_busbw_gbps\":%.3f,\"wrong\":%llu}\n",
             devs.size(), peak_alg, peak_bus, wrong_total);
    else
      printf("# peak algbw %.2f GB/s, peak busbw %.2f GB/s, wrong elements %llu\n", peak_alg, peak_bus, wrong_total);
    return wrong_total ? 1 : 0;
  } catch (const std::exception& e) {
    fprintf(stderr, "rccl_allreduce_bench: %s\n", e.what());
    return 3;
  }
}
