// Native GPU topology discovery for MI355X nodes (pybind11 module `_topo`).
//
// Reference: design.md:23-59 — the device plugin queries the P2P link type of every GPU pair via
// NVML (cgo FFI) at init; design.md:57-74 stores it in `map[uint]map[uint]gpuTopologyType`.
// MI355X-native replacement:
//   * amdsmi backend: amdsmi_topo_get_link_type (hops + INTERNAL/PCIE/XGMI), link weight,
//     min/max link bandwidth, NUMA node, P2P accessibility, compute/memory partition, xGMI link
//     status, enumeration info (render/card minors, HSA and HIP ids).  libamd_smi is dlopen'ed so
//     the module (and the sysfs backend) still loads on hosts without amdsmi.
//   * KFD sysfs backend: /sys/class/kfd/kfd/topology/nodes/*/{properties,io_links,p2p_links}.
//     Takes a root path so tests can point it at a synthetic tree.
// Both return the same dict schema, consumed by gpu_topology_on_k8s_amd/topology/discovery.py.
#include <amd_smi/amdsmi.h>
#include <dirent.h>
#include <dlfcn.h>
#ifndef GTK_TOPO_NO_PYTHON  // the sanitizer self-test (topo_selftest.cpp) includes this file without Python
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#ifndef GTK_TOPO_NO_PYTHON
namespace py = pybind11;
#endif

namespace {

// ------------------------------------------------------------------------------------------------
// Common result model
struct Dev {
  int index = 0;
  std::string uuid, bdf, partition = "SPX", memory_partition = "NPS1", model, gfx;
  int numa = 0, render_minor = -1, card = -1, kfd_node = -1, hip_id = -1, physical = -1;
  uint64_t vram = 0;
  int xgmi_links_up = -1, xgmi_links_total = -1;
  // RAS signals for the device plugin's health monitor (-1 = not readable: unsupported / no root)
  int64_t ecc_correctable = -1, ecc_uncorrectable = -1, ecc_deferred = -1;
  int bad_pages = -1, bad_page_threshold = -1;
  int cus = 0;
  bool healthy = true;
  uint64_t location = 0;  // domain<<16 | bdf: physical-package key
  // GPU<->CPU path (PCI sysfs): cores local to the device's socket, and the trained PCIe link as a
  // fraction of its capability (speed x width; -1 = unreadable).  A link that trained at x8 or a
  // lower generation is a worse CPU-affinity choice for the same xGMI position (design.md:144-145).
  std::string cpulist;
  double pcie_link_ratio = -1.0;
};

// RDMA NIC (RoCE / InfiniBand verbs device) and its PCIe distance class to every GPU: multi-node
// RCCL traffic should leave through the NIC behind the GPU's own PCIe switch.
struct Nic {
  std::string name, bdf, netdev, state;
  int numa = -1;
  double rate_gbps = 0.0;
};

struct Result {
  std::string source;
  std::vector<Dev> devs;
  std::vector<Nic> nics;
  std::vector<std::vector<int>> gpu_nic;  // [gpu][nic] PCIe class: 1 PIX, 2 PXB, 3 PHB, 4 NODE, 5 SYS, 0 unknown
  std::vector<std::vector<int>> link_type, hops;  // link_type uses LinkType of model.py
  std::vector<std::vector<double>> weight, min_bw, max_bw;
  std::vector<std::vector<int>> p2p;
  std::map<int, std::vector<int>> numa_distance;  // NUMA node -> SLIT distances to every node
  std::vector<std::string> warnings;
};

// LinkType values mirrored from gpu_topology_on_k8s_amd/topology/model.py
enum : int { LT_SELF = 0, LT_INTERNAL = 1, LT_XGMI = 2, LT_PCIE = 3, LT_PCIE_SYS = 4, LT_UNKNOWN = 5 };

void init_mats(Result& r) {
  const size_t n = r.devs.size();
  r.link_type.assign(n, std::vector<int>(n, LT_UNKNOWN));
  r.hops.assign(n, std::vector<int>(n, 0));
  r.weight.assign(n, std::vector<double>(n, 0.0));
  r.min_bw.assign(n, std::vector<double>(n, 0.0));
  r.max_bw.assign(n, std::vector<double>(n, 0.0));
  r.p2p.assign(n, std::vector<int>(n, 0));
  for (size_t i = 0; i < n; ++i) {
    r.link_type[i][i] = LT_SELF;
    r.p2p[i][i] = 1;
  }
}

void assign_physical(Result& r) {
  std::map<uint64_t, int> pkg;
  for (auto& d : r.devs) {
    auto it = pkg.find(d.location);
    if (it == pkg.end()) it = pkg.emplace(d.location, (int)pkg.size()).first;
    d.physical = it->second;
  }
  // XCPs of one package: INTERNAL links regardless of what the backend reported
  for (size_t i = 0; i < r.devs.size(); ++i)
    for (size_t j = 0; j < r.devs.size(); ++j)
      if (i != j && r.devs[i].physical == r.devs[j].physical) {
        r.link_type[i][j] = LT_INTERNAL;
        r.hops[i][j] = 0;
        r.p2p[i][j] = 1;
      }
}

#ifndef GTK_TOPO_NO_PYTHON
py::dict to_py(const Result& r) {
  py::list gpus;
  for (const auto& d : r.devs) {
    py::dict g;
    g["index"] = d.index;
    g["uuid"] = d.uuid;
    g["bdf"] = d.bdf;
    g["numa"] = d.numa;
    g["render_minor"] = d.render_minor;
    g["card"] = d.card;
    g["kfd_node"] = d.kfd_node;
    g["hip_id"] = d.hip_id;
    g["physical"] = d.physical;
    g["partition"] = d.partition;
    g["memory_partition"] = d.memory_partition;
    g["model"] = d.model;
    g["gfx"] = d.gfx;
    g["vram_bytes"] = d.vram;
    g["healthy"] = d.healthy;
    g["xgmi_links_up"] = d.xgmi_links_up;
    g["xgmi_links_total"] = d.xgmi_links_total;
    g["ecc_correctable"] = d.ecc_correctable;
    g["ecc_uncorrectable"] = d.ecc_uncorrectable;
    g["ecc_deferred"] = d.ecc_deferred;
    g["bad_pages"] = d.bad_pages;
    g["bad_page_threshold"] = d.bad_page_threshold;
    g["cus"] = d.cus;
    g["cpu_affinity"] = d.cpulist;
    g["pcie_link_ratio"] = d.pcie_link_ratio;
    gpus.append(g);
  }
  py::dict out;
  out["source"] = r.source;
  out["gpus"] = gpus;
  out["link_type"] = r.link_type;
  out["hops"] = r.hops;
  out["weight"] = r.weight;
  out["min_bw_mbps"] = r.min_bw;
  out["max_bw_mbps"] = r.max_bw;
  out["p2p"] = r.p2p;
  py::dict nd;
  for (const auto& kv : r.numa_distance) nd[py::int_(kv.first)] = kv.second;
  out["numa_distance"] = nd;
  py::list nics;
  for (const auto& n : r.nics) {
    py::dict d;
    d["name"] = n.name;
    d["bdf"] = n.bdf;
    d["netdev"] = n.netdev;
    d["state"] = n.state;
    d["numa"] = n.numa;
    d["rate_gbps"] = n.rate_gbps;
    nics.append(d);
  }
  out["nics"] = nics;
  out["gpu_nic"] = r.gpu_nic;
  out["warnings"] = r.warnings;
  return out;
}
#endif

std::string fmt_bdf(uint64_t domain, uint64_t bus, uint64_t dev, uint64_t fn) {
  char buf[32];
  snprintf(buf, sizeof(buf), "%04llx:%02llx:%02llx.%llx", (unsigned long long)domain, (unsigned long long)bus,
           (unsigned long long)dev, (unsigned long long)fn);
  return buf;
}

// ------------------------------------------------------------------------------------------------
// amdsmi backend (dlopen)

// a fixed-size char field a library filled: at most `cap` bytes, whether or not it wrote the NUL
template <size_t N>
std::string field_str(const char (&f)[N]) {
  return std::string(f, strnlen(f, N));
}

struct AmdSmi {
  void* h = nullptr;
// decltype of the declared prototypes: no link-time dependency on libamd_smi
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) get_socket_handles = nullptr;
  decltype(&amdsmi_get_processor_handles) get_processor_handles = nullptr;
  decltype(&amdsmi_get_processor_type) get_processor_type = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) get_bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) get_uuid = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) get_enum = nullptr;
  decltype(&amdsmi_topo_get_numa_node_number) get_numa = nullptr;
  decltype(&amdsmi_topo_get_link_weight) get_weight = nullptr;
  decltype(&amdsmi_get_minmax_bandwidth_between_processors) get_minmax = nullptr;
  decltype(&amdsmi_topo_get_link_type) get_link_type = nullptr;
  decltype(&amdsmi_is_P2P_accessible) is_p2p = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) get_cpart = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) get_mpart = nullptr;
  decltype(&amdsmi_get_gpu_asic_info) get_asic = nullptr;
  decltype(&amdsmi_get_gpu_memory_total) get_mem_total = nullptr;
  decltype(&amdsmi_get_gpu_xgmi_link_status) get_xgmi_status = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) get_ecc_total = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_info) get_bad_pages = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_threshold) get_bad_page_threshold = nullptr;
  decltype(&amdsmi_init_gpu_event_notification) evt_init = nullptr;
  decltype(&amdsmi_set_gpu_event_notification_mask) evt_mask = nullptr;
  decltype(&amdsmi_get_gpu_event_notification) evt_get = nullptr;
  decltype(&amdsmi_stop_gpu_event_notification) evt_stop = nullptr;
  // partition control (topology/partition.py): read the modes a package offers, switch them
  decltype(&amdsmi_get_gpu_accelerator_partition_profile_config) get_profiles = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition_config) get_mpart_cfg = nullptr;
  decltype(&amdsmi_set_gpu_compute_partition) set_cpart = nullptr;
  decltype(&amdsmi_set_gpu_memory_partition) set_mpart = nullptr;
  decltype(&amdsmi_gpu_driver_reload) driver_reload = nullptr;

  template <class F>
  void bind(F& f, const char* sym, bool required) {
    f = reinterpret_cast<F>(dlsym(h, sym));
    if (!f && required) throw std::runtime_error(std::string("amdsmi symbol missing: ") + sym);
  }

  explicit AmdSmi(const std::string& path) {
    h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) throw std::runtime_error(std::string("dlopen amdsmi failed: ") + dlerror());
    bind(init, "amdsmi_init", true);
    bind(shut_down, "amdsmi_shut_down", true);
    bind(get_socket_handles, "amdsmi_get_socket_handles", true);
    bind(get_processor_handles, "amdsmi_get_processor_handles", true);
    bind(get_processor_type, "amdsmi_get_processor_type", true);
    bind(get_bdf, "amdsmi_get_gpu_device_bdf", true);
    bind(get_uuid, "amdsmi_get_gpu_device_uuid", false);
    bind(get_enum, "amdsmi_get_gpu_enumeration_info", false);
    bind(get_numa, "amdsmi_topo_get_numa_node_number", false);
    bind(get_weight, "amdsmi_topo_get_link_weight", false);
    bind(get_minmax, "amdsmi_get_minmax_bandwidth_between_processors", false);
    bind(get_link_type, "amdsmi_topo_get_link_type", true);
    bind(is_p2p, "amdsmi_is_P2P_accessible", false);
    bind(get_cpart, "amdsmi_get_gpu_compute_partition", false);
    bind(get_mpart, "amdsmi_get_gpu_memory_partition", false);
    bind(get_asic, "amdsmi_get_gpu_asic_info", false);
    bind(get_mem_total, "amdsmi_get_gpu_memory_total", false);
    bind(get_xgmi_status, "amdsmi_get_gpu_xgmi_link_status", false);
    bind(get_ecc_total, "amdsmi_get_gpu_total_ecc_count", false);
    bind(get_bad_pages, "amdsmi_get_gpu_bad_page_info", false);
    bind(get_bad_page_threshold, "amdsmi_get_gpu_bad_page_threshold", false);
    bind(evt_init, "amdsmi_init_gpu_event_notification", false);
    bind(evt_mask, "amdsmi_set_gpu_event_notification_mask", false);
    bind(evt_get, "amdsmi_get_gpu_event_notification", false);
    bind(evt_stop, "amdsmi_stop_gpu_event_notification", false);
    bind(get_profiles, "amdsmi_get_gpu_accelerator_partition_profile_config", false);
    bind(get_mpart_cfg, "amdsmi_get_gpu_memory_partition_config", false);
    bind(set_cpart, "amdsmi_set_gpu_compute_partition", false);
    bind(set_mpart, "amdsmi_set_gpu_memory_partition", false);
    bind(driver_reload, "amdsmi_gpu_driver_reload", false);
  }
  ~AmdSmi() {
    if (h) dlclose(h);
  }
};

// amdsmi_init / amdsmi_shut_down keep a process-wide reference count and handle table: the device
// plugin's health pass (discovery) and its GPU-event thread must not interleave them.  Every amdsmi
// session in this module runs under this lock (an event poll holds it for at most its timeout).
std::mutex g_amdsmi_mu;

Result discover_amdsmi_impl(const std::string& lib) {
  std::lock_guard<std::mutex> guard(g_amdsmi_mu);
  AmdSmi s(lib);
  amdsmi_status_t st = s.init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: status " + std::to_string((int)st));
  struct Closer {
    AmdSmi& s;
    ~Closer() { s.shut_down(); }
  } closer{s};

  Result r;
  r.source = "amdsmi";
  uint32_t nsock = 0;
  if (s.get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("socket count");
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock && s.get_socket_handles(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS)
    throw std::runtime_error("socket handles");
  std::vector<amdsmi_processor_handle> handles;
  for (auto sk : socks) {
    uint32_t np = 0;
    if (s.get_processor_handles(sk, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    if (np && s.get_processor_handles(sk, &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (auto p : ph) {
      processor_type_t t;
      if (s.get_processor_type(p, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU) handles.push_back(p);
    }
  }
  std::vector<Dev> devs(handles.size());
  for (size_t i = 0; i < handles.size(); ++i) {
    Dev& d = devs[i];
    auto h = handles[i];
    amdsmi_bdf_t bdf{};
    if (s.get_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
      d.bdf = fmt_bdf(bdf.domain_number, bdf.bus_number, bdf.device_number, bdf.function_number);
      d.location = ((uint64_t)bdf.domain_number << 16) | ((uint64_t)bdf.bus_number << 8) | ((uint64_t)bdf.device_number << 3);
    }
    if (s.get_uuid) {
      char buf[AMDSMI_MAX_STRING_LENGTH] = {0};
      unsigned int len = sizeof(buf);
      if (s.get_uuid(h, &len, buf) == AMDSMI_STATUS_SUCCESS) d.uuid = field_str(buf);
    }
    if (s.get_enum) {
      amdsmi_enumeration_info_t e{};
      if (s.get_enum(h, &e) == AMDSMI_STATUS_SUCCESS) {
        d.render_minor = (int)e.drm_render;
        d.card = (int)e.drm_card;
        d.kfd_node = (int)e.hsa_id;
        d.hip_id = (int)e.hip_id;
        if (d.uuid.empty()) d.uuid = field_str(e.hip_uuid);
      }
    }
    if (s.get_numa) {
      uint32_t nn = 0;
      if (s.get_numa(h, &nn) == AMDSMI_STATUS_SUCCESS) d.numa = (int)nn;
    }
    if (s.get_cpart) {
      char buf[64] = {0};
      if (s.get_cpart(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS && buf[0]) d.partition = field_str(buf);
    }
    if (s.get_mpart) {
      char buf[64] = {0};
      if (s.get_mpart(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS && buf[0]) d.memory_partition = field_str(buf);
    }
    if (s.get_asic) {
      amdsmi_asic_info_t a{};
      if (s.get_asic(h, &a) == AMDSMI_STATUS_SUCCESS) {
        d.model = field_str(a.market_name);
        if (a.num_of_compute_units != 0xFFFFFFFFu) d.cus = (int)a.num_of_compute_units;
        if (a.target_graphics_version != 0xFFFFFFFFFFFFFFFFull) {
          char gb[32];
          snprintf(gb, sizeof(gb), "gfx%llx", (unsigned long long)a.target_graphics_version);
          d.gfx = gb;
        }
      }
    }
    if (s.get_mem_total) {
      uint64_t tot = 0;
      if (s.get_mem_total(h, AMDSMI_MEM_TYPE_VRAM, &tot) == AMDSMI_STATUS_SUCCESS) d.vram = tot;
    }
    if (s.get_xgmi_status) {
      amdsmi_xgmi_link_status_t ls{};
      if (s.get_xgmi_status(h, &ls) == AMDSMI_STATUS_SUCCESS) {
        int up = 0;
        for (uint32_t l = 0; l < ls.total_links && l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l)
          up += ls.status[l] == AMDSMI_XGMI_LINK_UP;
        d.xgmi_links_up = up;
        d.xgmi_links_total = (int)std::min<uint32_t>(ls.total_links, AMDSMI_MAX_NUM_XGMI_LINKS);
      }
    }
    if (s.get_ecc_total) {
      amdsmi_error_count_t ec{};
      if (s.get_ecc_total(h, &ec) == AMDSMI_STATUS_SUCCESS) {
        d.ecc_correctable = (int64_t)ec.correctable_count;
        d.ecc_uncorrectable = (int64_t)ec.uncorrectable_count;
        d.ecc_deferred = (int64_t)ec.deferred_count;
      }
    }
    if (s.get_bad_pages) {
      uint32_t np = 0;
      if (s.get_bad_pages(h, &np, nullptr) == AMDSMI_STATUS_SUCCESS) d.bad_pages = (int)np;
    }
    if (s.get_bad_page_threshold) {
      uint32_t th = 0;
      if (s.get_bad_page_threshold(h, &th) == AMDSMI_STATUS_SUCCESS) d.bad_page_threshold = (int)th;
    }
  }
  // Order by HIP id when available (so index == HIP ordinal with no HIP_VISIBLE_DEVICES)
  std::vector<size_t> order(devs.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    int ka = devs[a].hip_id >= 0 ? devs[a].hip_id : 1 << 20;
    int kb = devs[b].hip_id >= 0 ? devs[b].hip_id : 1 << 20;
    return ka < kb;
  });
  for (size_t i = 0; i < order.size(); ++i) {
    r.devs.push_back(devs[order[i]]);
    r.devs.back().index = (int)i;
  }
  init_mats(r);
  const size_t n = r.devs.size();
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      if (i == j) continue;
      auto a = handles[order[i]], b = handles[order[j]];
      uint64_t hops = 0;
      amdsmi_link_type_t lt;
      if (s.get_link_type(a, b, &hops, &lt) == AMDSMI_STATUS_SUCCESS) {
        r.hops[i][j] = (int)hops;
        switch (lt) {
          case AMDSMI_LINK_TYPE_INTERNAL: r.link_type[i][j] = LT_INTERNAL; break;
          case AMDSMI_LINK_TYPE_XGMI: r.link_type[i][j] = LT_XGMI; break;
          case AMDSMI_LINK_TYPE_PCIE:
            r.link_type[i][j] = (r.devs[i].numa != r.devs[j].numa) ? LT_PCIE_SYS : LT_PCIE;
            break;
          default: r.link_type[i][j] = LT_UNKNOWN;
        }
      } else {
        r.warnings.push_back("link_type(" + std::to_string(i) + "," + std::to_string(j) + ") unavailable");
      }
      uint64_t w = 0;
      if (s.get_weight && s.get_weight(a, b, &w) == AMDSMI_STATUS_SUCCESS) r.weight[i][j] = (double)w;
      uint64_t mn = 0, mx = 0;
      if (s.get_minmax && s.get_minmax(a, b, &mn, &mx) == AMDSMI_STATUS_SUCCESS) {
        r.min_bw[i][j] = (double)mn;
        r.max_bw[i][j] = (double)mx;
      }
      bool acc = false;
      if (s.is_p2p && s.is_p2p(a, b, &acc) == AMDSMI_STATUS_SUCCESS) r.p2p[i][j] = acc ? 1 : 0;
    }
  assign_physical(r);
  return r;
}

// ------------------------------------------------------------------------------------------------
// Partition control: the hardware tier of Gaia's GPU virtualization (paper p.3 §III.A; SURVEY.md B3,
// B8: on MI355X a fraction of a GPU is an XCP of a CPX/DPX/QPX package, with NPS memory partitions).
// Discovery reads the modes; these read what each package OFFERS and switch it.  Partition settings
// belong to the package, so each call goes through the first processor (XCP) of every socket.
const char* accel_name(amdsmi_accelerator_partition_type_t t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_PARTITION_SPX: return "SPX";
    case AMDSMI_ACCELERATOR_PARTITION_DPX: return "DPX";
    case AMDSMI_ACCELERATOR_PARTITION_TPX: return "TPX";
    case AMDSMI_ACCELERATOR_PARTITION_QPX: return "QPX";
    case AMDSMI_ACCELERATOR_PARTITION_CPX: return "CPX";
    default: return "";
  }
}

bool compute_type(const std::string& m, amdsmi_compute_partition_type_t* t) {
  static const std::map<std::string, amdsmi_compute_partition_type_t> k = {
      {"SPX", AMDSMI_COMPUTE_PARTITION_SPX}, {"DPX", AMDSMI_COMPUTE_PARTITION_DPX}, {"TPX", AMDSMI_COMPUTE_PARTITION_TPX},
      {"QPX", AMDSMI_COMPUTE_PARTITION_QPX}, {"CPX", AMDSMI_COMPUTE_PARTITION_CPX}};
  auto it = k.find(m);
  if (it == k.end()) return false;
  *t = it->second;
  return true;
}

bool memory_type(const std::string& m, amdsmi_memory_partition_type_t* t) {
  static const std::map<std::string, amdsmi_memory_partition_type_t> k = {
      {"NPS1", AMDSMI_MEMORY_PARTITION_NPS1}, {"NPS2", AMDSMI_MEMORY_PARTITION_NPS2},
      {"NPS4", AMDSMI_MEMORY_PARTITION_NPS4}, {"NPS8", AMDSMI_MEMORY_PARTITION_NPS8}};
  auto it = k.find(m);
  if (it == k.end()) return false;
  *t = it->second;
  return true;
}

std::vector<std::string> nps_modes(amdsmi_nps_caps_t c) {
  std::vector<std::string> out;
  if (c.nps_flags.nps1_cap) out.push_back("NPS1");
  if (c.nps_flags.nps2_cap) out.push_back("NPS2");
  if (c.nps_flags.nps4_cap) out.push_back("NPS4");
  if (c.nps_flags.nps8_cap) out.push_back("NPS8");
  return out;
}

// one amdsmi session: the first GPU processor of every socket (= package), in socket order
struct Session {
  AmdSmi s;
  std::vector<amdsmi_processor_handle> pkg;
  std::vector<int> xcps;  // GPU processors per package
  explicit Session(const std::string& lib) : s(lib) {
    amdsmi_status_t st = s.init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: status " + std::to_string((int)st));
    uint32_t nsock = 0;
    if (s.get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) {
      s.shut_down();
      throw std::runtime_error("socket count");
    }
    std::vector<amdsmi_socket_handle> socks(nsock);
    if (nsock && s.get_socket_handles(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS) nsock = 0;
    nsock = std::min<uint32_t>(nsock, (uint32_t)socks.size());
    for (uint32_t k = 0; k < nsock; ++k) {
      uint32_t np = 0;
      if (s.get_processor_handles(socks[k], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      if (s.get_processor_handles(socks[k], &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
      amdsmi_processor_handle first = nullptr;
      int n = 0;
      for (auto p : ph) {
        processor_type_t t;
        if (s.get_processor_type(p, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU) {
          if (!first) first = p;
          ++n;
        }
      }
      if (first) {
        pkg.push_back(first);
        xcps.push_back(n);
      }
    }
  }
  ~Session() { s.shut_down(); }
  std::string bdf(amdsmi_processor_handle h) {
    amdsmi_bdf_t b{};
    if (s.get_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return "";
    return fmt_bdf(b.domain_number, b.bus_number, b.device_number, 0);  // the package: function 0
  }
};

struct PartInfo {
  std::string bdf, compute, memory;
  int xcps = 0;
  std::vector<std::string> compute_modes, memory_modes;
};

std::vector<PartInfo> partition_info_impl(const std::string& lib) {
  std::lock_guard<std::mutex> guard(g_amdsmi_mu);
  Session ss(lib);
  AmdSmi& s = ss.s;
  std::vector<PartInfo> out;
  for (size_t k = 0; k < ss.pkg.size(); ++k) {
    auto h = ss.pkg[k];
    PartInfo p;
    p.bdf = ss.bdf(h);
    p.xcps = ss.xcps[k];
    char buf[64] = {0};
    if (s.get_cpart && s.get_cpart(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) p.compute = field_str(buf);
    std::memset(buf, 0, sizeof(buf));
    if (s.get_mpart && s.get_mpart(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) p.memory = field_str(buf);
    if (s.get_profiles) {
      // a few KiB per profile: on the heap, not the stack
      auto cfg = std::make_unique<amdsmi_accelerator_partition_profile_config_t>();
      std::memset(cfg.get(), 0, sizeof(*cfg));
      if (s.get_profiles(h, cfg.get()) == AMDSMI_STATUS_SUCCESS)
        for (uint32_t i = 0; i < cfg->num_profiles && i < AMDSMI_MAX_ACCELERATOR_PROFILE; ++i) {
          const char* n = accel_name(cfg->profiles[i].profile_type);
          if (*n && std::find(p.compute_modes.begin(), p.compute_modes.end(), n) == p.compute_modes.end())
            p.compute_modes.push_back(n);
        }
    }
    if (s.get_mpart_cfg) {
      amdsmi_memory_partition_config_t mc;
      std::memset(&mc, 0, sizeof(mc));
      if (s.get_mpart_cfg(h, &mc) == AMDSMI_STATUS_SUCCESS) p.memory_modes = nps_modes(mc.partition_caps);
    }
    out.push_back(p);
  }
  return out;
}

// One step of a partition change on every package: ("compute"|"memory", mode) -> per package
// (bdf, amdsmi status).  A fresh session per step: a compute-partition switch re-enumerates the
// package's processors, so handles of an earlier session are not reused.
std::vector<std::pair<std::string, int>> set_partition_step_impl(const std::string& lib, const std::string& what,
                                                                 const std::string& mode) {
  std::lock_guard<std::mutex> guard(g_amdsmi_mu);
  Session ss(lib);
  AmdSmi& s = ss.s;
  std::vector<std::pair<std::string, int>> out;
  if (what == "compute") {
    amdsmi_compute_partition_type_t t;
    if (!compute_type(mode, &t)) throw std::invalid_argument("unknown compute partition " + mode);
    if (!s.set_cpart) throw std::runtime_error("amdsmi_set_gpu_compute_partition not available in " + lib);
    for (auto h : ss.pkg) out.emplace_back(ss.bdf(h), (int)s.set_cpart(h, t));
  } else if (what == "memory") {
    amdsmi_memory_partition_type_t t;
    if (!memory_type(mode, &t)) throw std::invalid_argument("unknown memory partition " + mode);
    if (!s.set_mpart) throw std::runtime_error("amdsmi_set_gpu_memory_partition not available in " + lib);
    for (auto h : ss.pkg) out.emplace_back(ss.bdf(h), (int)s.set_mpart(h, t));
  } else {
    throw std::invalid_argument("step must be 'compute' or 'memory'");
  }
  return out;
}

// amdgpu driver reload (a memory-partition change takes effect only after it; every GPU process of
// the node must be gone).  -> amdsmi status
int driver_reload_impl(const std::string& lib) {
  std::lock_guard<std::mutex> guard(g_amdsmi_mu);
  Session ss(lib);
  if (!ss.s.driver_reload) throw std::runtime_error("amdsmi_gpu_driver_reload not available in " + lib);
  return (int)ss.s.driver_reload();
}

// ------------------------------------------------------------------------------------------------
// GPU event notification (amdsmi): resets, VM faults, thermal throttling as they happen, instead of
// waiting for the next RAS poll (SURVEY.md §5.3 failure detection).  The device plugin polls this
// on its own thread; events name the device by PCI address.
const char* event_name(amdsmi_evt_notification_type_t e) {
  switch (e) {
    case AMDSMI_EVT_NOTIF_VMFAULT: return "VMFAULT";
    case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: return "THERMAL_THROTTLE";
    case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: return "GPU_PRE_RESET";
    case AMDSMI_EVT_NOTIF_GPU_POST_RESET: return "GPU_POST_RESET";
    case AMDSMI_EVT_NOTIF_MIGRATE_START: return "MIGRATE_START";
    case AMDSMI_EVT_NOTIF_MIGRATE_END: return "MIGRATE_END";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_START: return "PAGE_FAULT_START";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_END: return "PAGE_FAULT_END";
    case AMDSMI_EVT_NOTIF_QUEUE_EVICTION: return "QUEUE_EVICTION";
    case AMDSMI_EVT_NOTIF_QUEUE_RESTORE: return "QUEUE_RESTORE";
    case AMDSMI_EVT_NOTIF_UNMAP_FROM_GPU: return "UNMAP_FROM_GPU";
    case AMDSMI_EVT_NOTIF_PROCESS_START: return "PROCESS_START";
    case AMDSMI_EVT_NOTIF_PROCESS_END: return "PROCESS_END";
    default: return "NONE";
  }
}

class EventWatcher {
 public:
  EventWatcher(const std::string& lib, const std::vector<std::string>& kinds) : s_(lib) {
    std::lock_guard<std::mutex> guard(g_amdsmi_mu);
    try {
      open_locked(kinds);
    } catch (...) {
      close_locked();  // a half-open session: stop what was subscribed, drop the amdsmi reference
      throw;
    }
  }

  ~EventWatcher() { close(); }

  // Events collected for up to timeout_ms (returns early when some arrive): (bdf, kind, message).
  std::vector<std::tuple<std::string, std::string, std::string>> poll(int timeout_ms, uint32_t max_events) {
    std::vector<std::tuple<std::string, std::string, std::string>> out;
    std::lock_guard<std::mutex> guard(g_amdsmi_mu);
    if (handles_.empty()) return out;
    std::vector<amdsmi_evt_notification_data_t> buf(std::max<uint32_t>(1, max_events));
    uint32_t n = (uint32_t)buf.size();
    amdsmi_status_t st = s_.evt_get(timeout_ms, &n, buf.data());
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_NO_DATA) return out;
    for (uint32_t i = 0; i < n && i < buf.size(); ++i) {
      std::string bdf;
      for (size_t j = 0; j < handles_.size(); ++j)
        if (handles_[j] == buf[i].processor_handle) bdf = bdfs_[j];
      buf[i].message[AMDSMI_MAX_STRING_LENGTH - 1] = 0;
      out.emplace_back(bdf, event_name(buf[i].event), std::string(buf[i].message));
    }
    return out;
  }

  void close() {
    std::lock_guard<std::mutex> guard(g_amdsmi_mu);
    close_locked();
  }
  const std::vector<std::string>& bdfs() const { return bdfs_; }


 private:
  void open_locked(const std::vector<std::string>& kinds) {
    if (!s_.evt_init || !s_.evt_mask || !s_.evt_get || !s_.evt_stop)
      throw std::runtime_error("this amdsmi has no GPU event notification API");
    uint64_t mask = 0;
    for (const auto& k : kinds) {
      int id = -1;
      for (int e = AMDSMI_EVT_NOTIF_FIRST; e <= AMDSMI_EVT_NOTIF_LAST; ++e)
        if (k == event_name((amdsmi_evt_notification_type_t)e)) id = e;
      if (id < 0) throw std::invalid_argument("unknown GPU event kind: " + k);
      mask |= AMDSMI_EVENT_MASK_FROM_INDEX(id);
    }
    if (s_.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed");
    inited_ = true;
    uint32_t nsock = 0;
    if (s_.get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("socket count");
    std::vector<amdsmi_socket_handle> socks(nsock);
    if (nsock && s_.get_socket_handles(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("socket handles");
    for (auto sk : socks) {
      uint32_t np = 0;
      if (s_.get_processor_handles(sk, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      if (np && s_.get_processor_handles(sk, &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
      for (auto p : ph) {
        processor_type_t t;
        if (s_.get_processor_type(p, &t) != AMDSMI_STATUS_SUCCESS || t != AMDSMI_PROCESSOR_TYPE_AMD_GPU) continue;
        amdsmi_bdf_t b;
        std::string bdf;
        if (s_.get_bdf(p, &b) == AMDSMI_STATUS_SUCCESS) bdf = fmt_bdf(b.domain_number, b.bus_number, b.device_number, b.function_number);
        if (s_.evt_init(p) != AMDSMI_STATUS_SUCCESS) continue;  // e.g. no permission on this device
        handles_.push_back(p);
        bdfs_.push_back(bdf);
        if (s_.evt_mask(p, mask) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("event mask on " + bdf);
      }
    }
    if (handles_.empty()) throw std::runtime_error("no GPU accepted event notification");
  }
  void close_locked() {
    for (auto p : handles_) s_.evt_stop(p);
    handles_.clear();
    if (inited_) s_.shut_down();
    inited_ = false;
  }


  AmdSmi s_;
  bool inited_ = false;
  std::vector<amdsmi_processor_handle> handles_;
  std::vector<std::string> bdfs_;
};

// ------------------------------------------------------------------------------------------------
// KFD sysfs backend
std::map<std::string, std::string> read_props(const std::string& path) {
  std::map<std::string, std::string> m;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string k, v;
    if (ss >> k >> v) m[k] = v;
  }
  return m;
}

// whole-string decimal int (sysfs names such as "12", "node3", "card1" after their prefix); false for
// anything else, including values out of int range: a stray entry is skipped, not fatal
bool to_int(const std::string& s, int* out) {
  if (s.empty() || s.size() > 9 || !std::all_of(s.begin(), s.end(), ::isdigit)) return false;
  *out = (int)std::strtol(s.c_str(), nullptr, 10);
  return true;
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = opendir(path.c_str());
  if (!d) return out;
  while (auto* e = readdir(d)) {
    std::string n = e->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    bool na = !a.empty() && std::all_of(a.begin(), a.end(), ::isdigit);
    bool nb = !b.empty() && std::all_of(b.begin(), b.end(), ::isdigit);
    if (na && nb) return a.size() != b.size() ? a.size() < b.size() : a < b;  // numeric order, any length
    return a < b;
  });
  return out;
}

uint64_t as_u64(const std::map<std::string, std::string>& m, const std::string& k, uint64_t dflt = 0) {
  auto it = m.find(k);
  if (it == m.end()) return dflt;
  try {
    return std::stoull(it->second);
  } catch (...) {
    return dflt;
  }
}

std::string read_first_line(const std::string& path) {
  std::ifstream f(path);
  std::string s;
  std::getline(f, s);
  return s;
}

// "16.0 GT/s PCIe" -> 16.0 ; "32.0 GT/s" -> 32.0 ; unknown -> 0
double link_speed_gts(const std::string& s) {
  try {
    return std::stod(s);
  } catch (...) {
    return 0.0;
  }
}

std::string pci_dir(const std::string& pci_root, const std::string& bdf) {
  // XCP partitions of one package may carry function numbers with no PCI function behind them:
  // fall back to function 0 of the same bus/device
  std::string p = pci_root + "/" + bdf;
  if (!read_first_line(p + "/vendor").empty() || bdf.size() < 2) return p;
  return pci_root + "/" + bdf.substr(0, bdf.size() - 1) + "0";
}

// Local cpulist + PCIe link ratio per device, NUMA SLIT distances per node.
void read_host_affinity(Result& r, const std::string& pci_root, const std::string& node_root) {
  for (auto& d : r.devs) {
    if (d.bdf.empty() || pci_root.empty()) continue;
    const std::string dir = pci_dir(pci_root, d.bdf);
    d.cpulist = read_first_line(dir + "/local_cpulist");
    double cs = link_speed_gts(read_first_line(dir + "/current_link_speed"));
    double ms = link_speed_gts(read_first_line(dir + "/max_link_speed"));
    double cw = link_speed_gts(read_first_line(dir + "/current_link_width"));
    double mw = link_speed_gts(read_first_line(dir + "/max_link_width"));
    if (cs > 0 && ms > 0 && cw > 0 && mw > 0) d.pcie_link_ratio = std::min(1.0, (cs * cw) / (ms * mw));
  }
  if (node_root.empty()) return;
  for (const auto& e : list_dir(node_root)) {
    if (e.rfind("node", 0) != 0 || e.size() < 5 || !std::all_of(e.begin() + 4, e.end(), ::isdigit)) continue;
    std::istringstream ss(read_first_line(node_root + "/" + e + "/distance"));
    std::vector<int> dist;
    int v;
    while (ss >> v) dist.push_back(v);
    int nn = 0;
    if (!dist.empty() && to_int(e.substr(4), &nn)) r.numa_distance[nn] = dist;
  }
}

// PCI path of a device below /sys/devices: ["pci0000:00", "0000:00:01.1", ..., "<bdf>"] (empty if unknown)
std::vector<std::string> pci_path(const std::string& link) {
  char buf[4096];
  if (!realpath(link.c_str(), buf)) return {};
  std::vector<std::string> parts;
  std::stringstream ss(buf);
  std::string item;
  bool in = false;
  while (std::getline(ss, item, '/')) {
    if (!in && item.rfind("pci", 0) == 0 && item.find(':') != std::string::npos) in = true;
    if (in && !item.empty()) parts.push_back(item);
  }
  return parts;
}

// The reference's PCIe taxonomy (design.md:31-47, nvidia-smi topo -m) for a GPU-NIC pair:
// PIX = behind one PCIe switch, PXB = several bridges below the same root port, PHB = through the host
// bridge, NODE = different root complexes of one NUMA node, SYS = across sockets.
int pcie_class(const std::vector<std::string>& a, const std::vector<std::string>& b, int numa_a, int numa_b) {
  if (a.empty() || b.empty()) return 0;
  if (a[0] != b[0]) return numa_a >= 0 && numa_a == numa_b ? 4 : 5;
  size_t l = 0;
  while (l < a.size() && l < b.size() && a[l] == b[l]) ++l;
  if (l <= 1) return 3;
  if (a.size() - l <= 2 && b.size() - l <= 2) return 1;
  return 2;
}

void read_nics(Result& r, const std::string& pci_root, const std::string& ib_root) {
  if (ib_root.empty()) return;
  std::vector<std::vector<std::string>> nic_paths;
  for (const auto& name : list_dir(ib_root)) {
    if (name.empty() || name[0] == '.') continue;
    const std::string dev = ib_root + "/" + name + "/device";
    auto path = pci_path(dev);
    if (path.empty()) continue;
    Nic n;
    n.name = name;
    n.bdf = path.back();
    const std::string numa = read_first_line(dev + "/numa_node");
    if (!numa.empty()) n.numa = std::atoi(numa.c_str());
    n.state = read_first_line(ib_root + "/" + name + "/ports/1/state");  // e.g. "4: ACTIVE"
    n.rate_gbps = std::atof(read_first_line(ib_root + "/" + name + "/ports/1/rate").c_str());  // "400 Gb/sec (4X NDR)"
    for (const auto& nd : list_dir(dev + "/net"))
      if (!nd.empty() && nd[0] != '.') n.netdev = nd;
    r.nics.push_back(n);
    nic_paths.push_back(path);
  }
  r.gpu_nic.assign(r.devs.size(), std::vector<int>(r.nics.size(), 0));
  for (size_t g = 0; g < r.devs.size(); ++g) {
    if (r.devs[g].bdf.empty() || pci_root.empty()) continue;
    auto gp = pci_path(pci_dir(pci_root, r.devs[g].bdf));
    for (size_t i = 0; i < r.nics.size(); ++i) r.gpu_nic[g][i] = pcie_class(gp, nic_paths[i], r.devs[g].numa, r.nics[i].numa);
  }
}

struct KfdLink {
  int from, to, type;
  double weight, min_bw, max_bw;
};

Result discover_sysfs_impl(const std::string& root, const std::string& drm_root) {
  Result r;
  r.source = "sysfs";
  const std::string nodes_dir = root + "/nodes";
  auto nodes = list_dir(nodes_dir);
  if (nodes.empty()) throw std::runtime_error("no KFD topology nodes under " + nodes_dir);
  std::map<int, std::map<std::string, std::string>> props;
  std::map<int, std::vector<KfdLink>> direct, indirect;
  std::map<int, bool> is_cpu;
  for (const auto& nd : nodes) {
    int id = 0;
    if (!to_int(nd, &id)) continue;  // not a KFD node directory
    auto p = read_props(nodes_dir + "/" + nd + "/properties");
    props[id] = p;
    is_cpu[id] = as_u64(p, "simd_count") == 0;
    for (const char* sub : {"io_links", "p2p_links"}) {
      std::string ld = nodes_dir + "/" + nd + "/" + sub;
      for (const auto& l : list_dir(ld)) {
        auto lp = read_props(ld + "/" + l + "/properties");
        KfdLink k{(int)as_u64(lp, "node_from", id), (int)as_u64(lp, "node_to", -1), (int)as_u64(lp, "type"),
                  (double)as_u64(lp, "weight"), (double)as_u64(lp, "min_bandwidth"), (double)as_u64(lp, "max_bandwidth")};
        (std::string(sub) == "io_links" ? direct : indirect)[id].push_back(k);
      }
    }
  }
  std::vector<int> gpu_nodes;
  for (auto& kv : props)
    if (!is_cpu[kv.first]) gpu_nodes.push_back(kv.first);
  std::map<int, int> idx_of;
  for (size_t i = 0; i < gpu_nodes.size(); ++i) {
    int nid = gpu_nodes[i];
    auto& p = props[nid];
    Dev d;
    d.index = (int)i;
    d.kfd_node = nid;
    d.hip_id = (int)i;
    d.render_minor = (int)as_u64(p, "drm_render_minor", (uint64_t)-1);
    uint64_t loc = as_u64(p, "location_id"), dom = as_u64(p, "domain");
    d.bdf = fmt_bdf(dom, (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 0x7);
    d.location = (dom << 16) | (loc & ~7ull);
    uint64_t uid = as_u64(p, "unique_id");
    if (uid) {
      char b[40];
      snprintf(b, sizeof(b), "GPU-%016llx", (unsigned long long)uid);
      d.uuid = b;
    }
    uint64_t gtv = as_u64(p, "gfx_target_version");
    if (gtv) {
      char b[32];
      snprintf(b, sizeof(b), "gfx%llu%llu%llx", (unsigned long long)(gtv / 10000), (unsigned long long)((gtv / 100) % 100),
               (unsigned long long)(gtv % 100));
      d.gfx = b;
    }
    d.cus = (int)(as_u64(p, "simd_count") / std::max<uint64_t>(1, as_u64(p, "simd_per_cu", 4)));
    d.vram = as_u64(p, "local_mem_size");
    d.model = d.gfx == "gfx950" ? "MI355X" : "";
    // NUMA: the CPU node this GPU's PCIe io_link lands on
    for (const auto& l : direct[nid])
      if (is_cpu.count(l.to) && is_cpu[l.to]) {
        d.numa = l.to;
        break;
      }
    int up = 0;
    for (const auto& l : direct[nid]) up += (l.type == 11);
    d.xgmi_links_up = up;
    d.xgmi_links_total = up;  // KFD lists only links that trained; amdsmi reports the down ones
    if (!drm_root.empty() && d.render_minor >= 0) {
      std::string dev = drm_root + "/renderD" + std::to_string(d.render_minor) + "/device/";
      std::string cp = read_first_line(dev + "current_compute_partition");
      std::string mp = read_first_line(dev + "current_memory_partition");
      if (!cp.empty()) d.partition = cp;
      if (!mp.empty()) d.memory_partition = mp;
      // RAS: amdgpu's per-block ras/<block>_err_count files ("ue: N" / "ce: M"), summed, and the
      // retired-page list ras/gpu_vram_bad_pages (one line per page)
      const std::string ras = dev + "ras/";
      for (const auto& f : list_dir(ras)) {
        if (f.size() < 10 || f.compare(f.size() - 10, 10, "_err_count") != 0) continue;
        std::ifstream in(ras + f);
        std::string key;
        uint64_t v = 0;
        while (in >> key >> v) {
          if (key == "ue:") d.ecc_uncorrectable = std::max<int64_t>(d.ecc_uncorrectable, 0) + (int64_t)v;
          if (key == "ce:") d.ecc_correctable = std::max<int64_t>(d.ecc_correctable, 0) + (int64_t)v;
        }
      }
      {
        std::ifstream bp(ras + "gpu_vram_bad_pages");
        if (bp) {
          int n = 0;
          std::string line;
          while (std::getline(bp, line))
            if (!line.empty()) ++n;
          d.bad_pages = n;
        }
      }
      // the card minor: first cardN directory under the device's drm/
      for (const auto& c : list_dir(dev + "drm")) {
        int cm = 0;
        if (c.rfind("card", 0) == 0 && to_int(c.substr(4), &cm)) {
          d.card = cm;
          break;
        }
      }
    }
    idx_of[nid] = (int)i;
    r.devs.push_back(d);
  }
  init_mats(r);
  const size_t n = r.devs.size();
  for (size_t i = 0; i < n; ++i) {
    int nid = gpu_nodes[i];
    for (size_t j = 0; j < n; ++j) {
      if (i == j) continue;
      int to = gpu_nodes[j];
      const KfdLink* best = nullptr;
      bool is_direct = false;
      for (const auto& l : direct[nid])
        if (l.to == to) {
          best = &l;
          is_direct = true;
        }
      if (!best)
        for (const auto& l : indirect[nid])
          if (l.to == to) best = &l;
      if (best) {
        r.weight[i][j] = best->weight;
        r.min_bw[i][j] = best->min_bw;
        r.max_bw[i][j] = best->max_bw;
        r.p2p[i][j] = 1;
        if (best->type == 11) {
          r.link_type[i][j] = LT_XGMI;
          r.hops[i][j] = is_direct ? 1 : 2;
        } else {
          bool cross = r.devs[i].numa != r.devs[j].numa;
          r.link_type[i][j] = cross ? LT_PCIE_SYS : LT_PCIE;
          r.hops[i][j] = cross ? 3 : 2;
        }
      } else {
        bool cross = r.devs[i].numa != r.devs[j].numa;
        r.link_type[i][j] = cross ? LT_PCIE_SYS : LT_PCIE;
        r.hops[i][j] = cross ? 3 : 2;
        r.warnings.push_back("no KFD link " + std::to_string(nid) + "->" + std::to_string(to) + ", assuming PCIe");
      }
    }
  }
  assign_physical(r);
  return r;
}

}  // namespace

#ifndef GTK_TOPO_NO_PYTHON
PYBIND11_MODULE(_topo, m) {
  m.doc() = "MI355X topology discovery: amdsmi (dlopen) and KFD sysfs backends";
  m.def(
      "discover_amdsmi",
      [](const std::string& lib, const std::string& pci_root, const std::string& node_root, const std::string& ib_root) {
        Result r;
        {
          py::gil_scoped_release nogil;
          r = discover_amdsmi_impl(lib);
          read_host_affinity(r, pci_root, node_root);
          read_nics(r, pci_root, ib_root);
        }
        return to_py(r);
      },
      py::arg("lib") = "libamd_smi.so", py::arg("pci_root") = "/sys/bus/pci/devices",
      py::arg("node_root") = "/sys/devices/system/node", py::arg("ib_root") = "/sys/class/infiniband");
  m.def(
      "discover_sysfs",
      [](const std::string& root, const std::string& drm_root, const std::string& pci_root, const std::string& node_root,
         const std::string& ib_root) {
        Result r;
        {
          py::gil_scoped_release nogil;
          r = discover_sysfs_impl(root, drm_root);
          read_host_affinity(r, pci_root, node_root);
          read_nics(r, pci_root, ib_root);
        }
        return to_py(r);
      },
      py::arg("root") = "/sys/class/kfd/kfd/topology", py::arg("drm_root") = "/sys/class/drm",
      py::arg("pci_root") = "/sys/bus/pci/devices", py::arg("node_root") = "/sys/devices/system/node",
      py::arg("ib_root") = "/sys/class/infiniband");
  m.def(
      "partition_info",
      [](const std::string& lib) {
        std::vector<PartInfo> v;
        {
          py::gil_scoped_release nogil;
          v = partition_info_impl(lib);
        }
        py::list out;
        for (const auto& p : v) {
          py::dict d;
          d["bdf"] = p.bdf;
          d["compute"] = p.compute;
          d["memory"] = p.memory;
          d["xcps"] = p.xcps;
          d["compute_modes"] = p.compute_modes;
          d["memory_modes"] = p.memory_modes;
          out.append(d);
        }
        return out;
      },
      py::arg("lib") = "libamd_smi.so",
      "per package (socket order): current compute / memory partition, XCPs, and the modes it offers (read-only)");
  m.def(
      "set_partition_step",
      [](const std::string& lib, const std::string& what, const std::string& mode) {
        py::gil_scoped_release nogil;
        return set_partition_step_impl(lib, what, mode);
      },
      py::arg("lib"), py::arg("what"), py::arg("mode"),
      "switch every package's compute or memory partition; -> [(package bdf, amdsmi status)]");
  m.def(
      "driver_reload",
      [](const std::string& lib) {
        py::gil_scoped_release nogil;
        return driver_reload_impl(lib);
      },
      py::arg("lib"), "reload the amdgpu driver (completes a memory-partition change); -> amdsmi status");
  py::class_<EventWatcher>(m, "EventWatcher")
      .def(py::init<const std::string&, const std::vector<std::string>&>(), py::arg("lib") = "libamd_smi.so",
           py::arg("kinds") = std::vector<std::string>{"GPU_PRE_RESET", "GPU_POST_RESET", "VMFAULT", "THERMAL_THROTTLE"})
      .def("poll",
           [](EventWatcher& w, int timeout_ms, uint32_t max_events) {
             std::vector<std::tuple<std::string, std::string, std::string>> ev;
             {
               py::gil_scoped_release nogil;
               ev = w.poll(timeout_ms, max_events);
             }
             return ev;
           },
           py::arg("timeout_ms") = 1000, py::arg("max_events") = 64)
      .def("close", &EventWatcher::close)
      .def_property_readonly("bdfs", &EventWatcher::bdfs);
  m.attr("HSA_IOLINK_TYPE_XGMI") = 11;
  m.attr("HSA_IOLINK_TYPE_PCIEXPRESS") = 2;
}
#endif  // GTK_TOPO_NO_PYTHON
