// Stand-in libamd_smi for CPU tests of the amdsmi backend of csrc/topo/topo_reader.cpp.
//
// The test box has one GPU, so the pairwise half of the amdsmi backend (link type / hops / weight /
// min-max bandwidth / P2P for every ordered pair, ordering by HIP id, partition packages, xGMI link
// status) never runs on hardware before the driver's 8-GPU scaling run — where bench.py's rank 0
// discovers the node through exactly this code.  This library implements the amdsmi entry points the
// reader dlopen()s, with the header's own prototypes (so a signature drift fails the build), for a
// configurable node:
//   FAKE_AMDSMI_GPUS        physical MI355X packages (default 8), sockets split 2 ways by NUMA
//   FAKE_AMDSMI_PARTITIONS  XCPs per package (1 = SPX, 8 = CPX)
//   FAKE_AMDSMI_HIP_ORDER   comma list: HIP id of each enumerated processor (default identity)
//   FAKE_AMDSMI_DOWN        "a-b": the xGMI link between packages a and b is down (PCIe, 2 hops)
//   FAKE_AMDSMI_EVENTS_FILE GPU event script: every line "<processor index> <event id> <message>" is
//                           delivered once by amdsmi_get_gpu_event_notification (lines appended while
//                           a watcher runs arrive on its next poll)
//   FAKE_AMDSMI_STATE       partition state file ("<xcps> <memory mode> <pending memory mode>"): when
//                           set, it overrides FAKE_AMDSMI_PARTITIONS at every amdsmi_init, and the
//                           partition setters write it, so a switch shows on the next session (as a
//                           real compute-partition switch re-enumerates the processors); a memory mode
//                           is pending until amdsmi_gpu_driver_reload, as on hardware
//   FAKE_AMDSMI_SET_STATUS  status every partition setter / the driver reload returns instead of acting
//                           (e.g. 10 = AMDSMI_STATUS_NO_PERM: the plugin is not privileged)
// Partition rules mirror MI300-class parts: SPX/DPX/QPX/CPX (no TPX), NPS1 always, NPS4 with CPX only.
// Built by gpu_topology_on_k8s_amd/_native/build.py (target fake_amdsmi); never loaded in production.
#include <amd_smi/amdsmi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Node {
  int pkgs = 8, parts = 1, down_a = -1, down_b = -1;
  std::string mem = "NPS1", mem_pending;
  std::vector<int> hip;
  int n() const { return pkgs * parts; }
};

Node g_node;
bool g_init = false;

int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}

void read_state() {
  const char* path = std::getenv("FAKE_AMDSMI_STATE");
  if (!path) return;
  std::ifstream f(path);
  int parts = 0;
  std::string mem, pending;
  if (f >> parts >> mem) {
    g_node.parts = parts;
    g_node.mem = mem;
    if (f >> pending && pending != "-") g_node.mem_pending = pending;
  }
}

bool write_state(int parts, const std::string& mem, const std::string& pending) {
  const char* path = std::getenv("FAKE_AMDSMI_STATE");
  if (!path) return false;
  std::ofstream f(path, std::ios::trunc);
  f << parts << " " << mem << " " << (pending.empty() ? "-" : pending) << "\n";
  return bool(f);
}

void load() {
  g_node = Node{};
  g_node.pkgs = env_int("FAKE_AMDSMI_GPUS", 8);
  g_node.parts = env_int("FAKE_AMDSMI_PARTITIONS", 1);
  read_state();
  const int n = g_node.n();
  g_node.hip.resize(n);
  for (int i = 0; i < n; ++i) g_node.hip[i] = i;
  if (const char* o = std::getenv("FAKE_AMDSMI_HIP_ORDER")) {
    std::string s(o);
    size_t pos = 0;
    for (int i = 0; i < n && pos <= s.size(); ++i) {
      size_t c = s.find(',', pos);
      g_node.hip[i] = std::atoi(s.substr(pos, c - pos).c_str());
      if (c == std::string::npos) break;
      pos = c + 1;
    }
  }
  if (const char* d = std::getenv("FAKE_AMDSMI_DOWN")) std::sscanf(d, "%d-%d", &g_node.down_a, &g_node.down_b);
}

// handles are 1-based indices: processor i <-> (void*)(i + 1); socket p <-> (void*)(0x10000 + p)
int idx(amdsmi_processor_handle h) {
  const intptr_t v = reinterpret_cast<intptr_t>(h) - 1;
  return (v >= 0 && v < g_node.n()) ? (int)v : -1;
}
int pkg(int i) { return i / g_node.parts; }
bool is_down(int a, int b) {
  const int pa = pkg(a), pb = pkg(b);
  return (pa == g_node.down_a && pb == g_node.down_b) || (pa == g_node.down_b && pb == g_node.down_a);
}

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  load();
  g_init = true;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  g_init = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* socket_count, amdsmi_socket_handle* socket_handles) {
  if (!g_init || !socket_count) return AMDSMI_STATUS_INVAL;
  if (!socket_handles) {
    *socket_count = (uint32_t)g_node.pkgs;
    return AMDSMI_STATUS_SUCCESS;
  }
  const uint32_t n = std::min<uint32_t>(*socket_count, (uint32_t)g_node.pkgs);
  for (uint32_t p = 0; p < n; ++p) socket_handles[p] = reinterpret_cast<amdsmi_socket_handle>((intptr_t)(0x10000 + p));
  *socket_count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle socket_handle, uint32_t* processor_count,
                                             amdsmi_processor_handle* processor_handles) {
  const intptr_t p = reinterpret_cast<intptr_t>(socket_handle) - 0x10000;
  if (!processor_count || p < 0 || p >= g_node.pkgs) return AMDSMI_STATUS_INVAL;
  if (!processor_handles) {
    *processor_count = (uint32_t)g_node.parts;
    return AMDSMI_STATUS_SUCCESS;
  }
  const uint32_t n = std::min<uint32_t>(*processor_count, (uint32_t)g_node.parts);
  for (uint32_t x = 0; x < n; ++x)
    processor_handles[x] = reinterpret_cast<amdsmi_processor_handle>((intptr_t)(p * g_node.parts + x + 1));
  *processor_count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle h, processor_type_t* t) {
  if (idx(h) < 0 || !t) return AMDSMI_STATUS_INVAL;
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  const int i = idx(h);
  if (i < 0 || !bdf) return AMDSMI_STATUS_INVAL;
  bdf->as_uint = 0;
  bdf->domain_number = 0;
  bdf->bus_number = (uint64_t)(0x05 + 0x10 * pkg(i));
  bdf->device_number = 0;
  bdf->function_number = (uint64_t)(i % g_node.parts);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* uuid_length, char* uuid) {
  const int i = idx(h);
  if (i < 0 || !uuid_length || !uuid) return AMDSMI_STATUS_INVAL;
  std::snprintf(uuid, *uuid_length, "fake-%02d-xcp%d", pkg(i), i % g_node.parts);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h, amdsmi_enumeration_info_t* info) {
  const int i = idx(h);
  if (i < 0 || !info) return AMDSMI_STATUS_INVAL;
  std::memset(info, 0, sizeof(*info));
  info->drm_render = (uint32_t)(128 + i);
  info->drm_card = (uint32_t)i;
  info->hsa_id = (uint32_t)(i + 2);
  info->hip_id = (uint32_t)g_node.hip[i];
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_numa_node_number(amdsmi_processor_handle h, uint32_t* numa) {
  const int i = idx(h);
  if (i < 0 || !numa) return AMDSMI_STATUS_INVAL;
  *numa = (uint32_t)(pkg(i) < (g_node.pkgs + 1) / 2 ? 0 : 1);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_weight(amdsmi_processor_handle a, amdsmi_processor_handle b, uint64_t* weight) {
  const int i = idx(a), j = idx(b);
  if (i < 0 || j < 0 || !weight) return AMDSMI_STATUS_INVAL;
  *weight = pkg(i) == pkg(j) ? 10 : (is_down(i, j) ? 40 : 15);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_minmax_bandwidth_between_processors(amdsmi_processor_handle a, amdsmi_processor_handle b,
                                                               uint64_t* min_bandwidth, uint64_t* max_bandwidth) {
  const int i = idx(a), j = idx(b);
  if (i < 0 || j < 0 || !min_bandwidth || !max_bandwidth) return AMDSMI_STATUS_INVAL;
  *min_bandwidth = 0;
  *max_bandwidth = pkg(i) == pkg(j) ? 0 : (is_down(i, j) ? 64000 : 76800);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_type(amdsmi_processor_handle a, amdsmi_processor_handle b, uint64_t* hops,
                                          amdsmi_link_type_t* type) {
  const int i = idx(a), j = idx(b);
  if (i < 0 || j < 0 || !hops || !type) return AMDSMI_STATUS_INVAL;
  if (pkg(i) == pkg(j)) {
    *hops = 0;
    *type = AMDSMI_LINK_TYPE_INTERNAL;
  } else if (is_down(i, j)) {
    *hops = 2;
    *type = AMDSMI_LINK_TYPE_PCIE;
  } else {
    *hops = 1;
    *type = AMDSMI_LINK_TYPE_XGMI;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_is_P2P_accessible(amdsmi_processor_handle a, amdsmi_processor_handle b, bool* accessible) {
  if (idx(a) < 0 || idx(b) < 0 || !accessible) return AMDSMI_STATUS_INVAL;
  *accessible = true;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle h, char* compute_partition, uint32_t len) {
  if (idx(h) < 0 || !compute_partition || len < 4) return AMDSMI_STATUS_INVAL;
  const char* name = g_node.parts == 8 ? "CPX" : g_node.parts == 4 ? "QPX" : g_node.parts == 2 ? "DPX" : "SPX";
  std::snprintf(compute_partition, len, "%s", name);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle h, char* memory_partition, uint32_t len) {
  if (idx(h) < 0 || !memory_partition || len < 5) return AMDSMI_STATUS_INVAL;
  std::snprintf(memory_partition, len, "%s", g_node.mem.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

// ---- partition control (no TPX; NPS4 only together with CPX)
amdsmi_status_t amdsmi_get_gpu_accelerator_partition_profile_config(amdsmi_processor_handle h,
                                                                    amdsmi_accelerator_partition_profile_config_t* cfg) {
  if (idx(h) < 0 || !cfg) return AMDSMI_STATUS_INVAL;
  const amdsmi_accelerator_partition_type_t types[] = {AMDSMI_ACCELERATOR_PARTITION_SPX, AMDSMI_ACCELERATOR_PARTITION_DPX,
                                                       AMDSMI_ACCELERATOR_PARTITION_QPX, AMDSMI_ACCELERATOR_PARTITION_CPX};
  const uint32_t parts[] = {1, 2, 4, 8};
  cfg->num_profiles = 4;
  cfg->default_profile_index = 0;
  for (uint32_t i = 0; i < 4; ++i) {
    amdsmi_accelerator_partition_profile_t& p = cfg->profiles[i];
    p.profile_type = types[i];
    p.num_partitions = parts[i];
    p.profile_index = i;
    p.memory_caps.nps_cap_mask = 0;
    p.memory_caps.nps_flags.nps1_cap = 1;
    p.memory_caps.nps_flags.nps4_cap = parts[i] == 8;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition_config(amdsmi_processor_handle h, amdsmi_memory_partition_config_t* cfg) {
  if (idx(h) < 0 || !cfg) return AMDSMI_STATUS_INVAL;
  cfg->partition_caps.nps_cap_mask = 0;
  cfg->partition_caps.nps_flags.nps1_cap = 1;
  cfg->partition_caps.nps_flags.nps4_cap = 1;
  cfg->mp_mode = g_node.mem == "NPS4" ? AMDSMI_MEMORY_PARTITION_NPS4 : AMDSMI_MEMORY_PARTITION_NPS1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_set_gpu_compute_partition(amdsmi_processor_handle h, amdsmi_compute_partition_type_t t) {
  if (idx(h) < 0) return AMDSMI_STATUS_INVAL;
  if (const char* st = std::getenv("FAKE_AMDSMI_SET_STATUS")) return (amdsmi_status_t)std::atoi(st);
  int parts = 0;
  switch (t) {
    case AMDSMI_COMPUTE_PARTITION_SPX: parts = 1; break;
    case AMDSMI_COMPUTE_PARTITION_DPX: parts = 2; break;
    case AMDSMI_COMPUTE_PARTITION_QPX: parts = 4; break;
    case AMDSMI_COMPUTE_PARTITION_CPX: parts = 8; break;
    default: return AMDSMI_STATUS_SETTING_UNAVAILABLE;
  }
  if (g_node.mem == "NPS4" && parts != 8) return AMDSMI_STATUS_SETTING_UNAVAILABLE;
  return write_state(parts, g_node.mem, g_node.mem_pending) ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NOT_SUPPORTED;
}

amdsmi_status_t amdsmi_set_gpu_memory_partition(amdsmi_processor_handle h, amdsmi_memory_partition_type_t t) {
  if (idx(h) < 0) return AMDSMI_STATUS_INVAL;
  if (const char* st = std::getenv("FAKE_AMDSMI_SET_STATUS")) return (amdsmi_status_t)std::atoi(st);
  // the session's view: a compute switch written by an earlier session is what the state file holds
  Node cur = g_node;
  read_state();
  const int parts = g_node.parts;
  g_node = cur;
  std::string m;
  if (t == AMDSMI_MEMORY_PARTITION_NPS1) m = "NPS1";
  else if (t == AMDSMI_MEMORY_PARTITION_NPS4 && parts == 8) m = "NPS4";
  else return AMDSMI_STATUS_SETTING_UNAVAILABLE;
  return write_state(parts, g_node.mem, m == g_node.mem ? "" : m) ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NOT_SUPPORTED;
}

amdsmi_status_t amdsmi_gpu_driver_reload(void) {
  if (const char* st = std::getenv("FAKE_AMDSMI_SET_STATUS")) return (amdsmi_status_t)std::atoi(st);
  Node cur = g_node;
  read_state();
  const int parts = g_node.parts;
  const std::string mem = g_node.mem_pending.empty() ? g_node.mem : g_node.mem_pending;
  g_node = cur;
  return write_state(parts, mem, "") ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NOT_SUPPORTED;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* info) {
  if (idx(h) < 0 || !info) return AMDSMI_STATUS_INVAL;
  std::memset(info, 0, sizeof(*info));
  std::snprintf(info->market_name, sizeof(info->market_name), "MI355X");
  info->num_of_compute_units = (uint32_t)(256 / g_node.parts);
  info->target_graphics_version = 0x950;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t, uint64_t* total) {
  if (idx(h) < 0 || !total) return AMDSMI_STATUS_INVAL;
  *total = (288ull << 30) / (uint64_t)g_node.parts;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h, amdsmi_xgmi_link_status_t* st) {
  const int i = idx(h);
  if (i < 0 || !st) return AMDSMI_STATUS_INVAL;
  std::memset(st, 0, sizeof(*st));
  st->total_links = AMDSMI_MAX_NUM_XGMI_LINKS;
  int link = 0;
  for (int p = 0; p < g_node.pkgs && link < AMDSMI_MAX_NUM_XGMI_LINKS; ++p) {
    if (p == pkg(i)) continue;
    const bool down = (pkg(i) == g_node.down_a && p == g_node.down_b) || (pkg(i) == g_node.down_b && p == g_node.down_a);
    st->status[link++] = down ? AMDSMI_XGMI_LINK_DOWN : AMDSMI_XGMI_LINK_UP;
  }
  for (; link < AMDSMI_MAX_NUM_XGMI_LINKS; ++link) st->status[link] = AMDSMI_XGMI_LINK_DISABLE;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h, amdsmi_error_count_t* ec) {
  if (idx(h) < 0 || !ec) return AMDSMI_STATUS_INVAL;
  std::memset(ec, 0, sizeof(*ec));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_info(amdsmi_processor_handle h, uint32_t* num_pages, amdsmi_retired_page_record_t*) {
  if (idx(h) < 0 || !num_pages) return AMDSMI_STATUS_INVAL;
  *num_pages = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_threshold(amdsmi_processor_handle h, uint32_t* threshold) {
  if (idx(h) < 0 || !threshold) return AMDSMI_STATUS_INVAL;
  *threshold = 128;
  return AMDSMI_STATUS_SUCCESS;
}

// ---- GPU event notification: scripted through FAKE_AMDSMI_EVENTS_FILE
namespace {
std::vector<uint64_t> g_evt_mask;
size_t g_evt_delivered = 0;

bool next_events(uint32_t cap, uint32_t* n, amdsmi_evt_notification_data_t* data) {
  const char* path = std::getenv("FAKE_AMDSMI_EVENTS_FILE");
  *n = 0;
  if (!path) return false;
  std::ifstream f(path);
  std::string line;
  size_t lineno = 0;
  while (*n < cap && std::getline(f, line)) {
    if (lineno++ < g_evt_delivered || line.empty()) continue;
    ++g_evt_delivered;
    int dev = -1, id = 0, off = 0;
    if (std::sscanf(line.c_str(), "%d %d %n", &dev, &id, &off) < 2 || dev < 0 || dev >= g_node.n()) continue;
    if (dev >= (int)g_evt_mask.size() || !(g_evt_mask[dev] & AMDSMI_EVENT_MASK_FROM_INDEX(id))) continue;
    amdsmi_evt_notification_data_t& d = data[(*n)++];
    d.processor_handle = reinterpret_cast<amdsmi_processor_handle>((intptr_t)dev + 1);
    d.event = (amdsmi_evt_notification_type_t)id;
    std::snprintf(d.message, sizeof(d.message), "%s", line.c_str() + off);
  }
  return *n > 0;
}
}  // namespace

amdsmi_status_t amdsmi_init_gpu_event_notification(amdsmi_processor_handle h) {
  if (!g_init || idx(h) < 0) return AMDSMI_STATUS_INVAL;
  if ((int)g_evt_mask.size() < g_node.n()) g_evt_mask.assign(g_node.n(), 0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_set_gpu_event_notification_mask(amdsmi_processor_handle h, uint64_t mask) {
  if (idx(h) < 0 || (int)g_evt_mask.size() <= idx(h)) return AMDSMI_STATUS_INVAL;
  g_evt_mask[idx(h)] = mask;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_event_notification(int timeout_ms, uint32_t* num_elem, amdsmi_evt_notification_data_t* data) {
  if (!num_elem || !data) return AMDSMI_STATUS_INVAL;
  const uint32_t cap = *num_elem;
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms));
  while (!next_events(cap, num_elem, data)) {
    if (std::chrono::steady_clock::now() >= until) return AMDSMI_STATUS_NO_DATA;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_stop_gpu_event_notification(amdsmi_processor_handle h) {
  if (idx(h) < 0) return AMDSMI_STATUS_INVAL;
  if (idx(h) < (int)g_evt_mask.size()) g_evt_mask[idx(h)] = 0;
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
