// libgpushare_gpuinfo implementation. See gpuinfo.h for the contract.
//
// Reference parity: nvml.Init/DeviceGetCount/GetUUID/GetMemoryInfo_v2 (nvidia.go:44-86,
// gpumanager.go:36-47) and the intended XID health stream (nvidia.go:97-153). Differences by
// design: every backend reports bytes (the reference mis-read bytes as MiB),
// per-device data is kept per device (no "first GPU wins" global), and errors are returned,
// never fatal (nvidia.go:17-21 called log.Fatalln).
#include "gpuinfo.h"

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "json_min.h"

namespace {

thread_local std::string g_err;
void set_err(const std::string& s) { g_err = s; }

template <size_t N>
void copy_str(char (&dst)[N], const std::string& s) {
  size_t n = std::min(s.size(), N - 1);
  memcpy(dst, s.data(), n);
  dst[n] = 0;
}

// ---------------------------------------------------------------------------------------
// sysfs helpers
// ---------------------------------------------------------------------------------------
bool read_file(const std::string& path, std::string* out, int* err = nullptr) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) {
    if (err) *err = errno;
    return false;
  }
  std::string s;
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  int e = ferror(f) ? errno : 0;
  fclose(f);
  if (e) {
    if (err) *err = e;
    return false;
  }
  *out = s;
  return true;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

std::string read_trim(const std::string& path) {
  std::string s;
  if (!read_file(path, &s)) return "";
  return trim(s);
}

std::map<std::string, std::string> parse_props(const std::string& s) {
  std::map<std::string, std::string> m;
  std::istringstream is(s);
  std::string line;
  while (std::getline(is, line)) {
    size_t sp = line.find_last_of(' ');
    if (sp == std::string::npos) continue;
    m[trim(line.substr(0, sp))] = trim(line.substr(sp + 1));
  }
  return m;
}

uint64_t to_u64(const std::string& s, uint64_t dflt = 0) {
  if (s.empty()) return dflt;
  errno = 0;
  char* end = nullptr;
  unsigned long long v = strtoull(s.c_str(), &end, 0);
  if (errno || end == s.c_str()) return dflt;
  return (uint64_t)v;
}

int64_t to_i64(const std::string& s, int64_t dflt) {
  if (s.empty()) return dflt;
  errno = 0;
  char* end = nullptr;
  long long v = strtoll(s.c_str(), &end, 0);
  if (errno || end == s.c_str()) return dflt;
  return (int64_t)v;
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> v;
  DIR* d = opendir(path.c_str());
  if (!d) return v;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    v.emplace_back(e->d_name);
  }
  closedir(d);
  return v;
}

std::vector<int> numeric_entries(const std::string& path) {
  std::vector<int> v;
  for (auto& s : list_dir(path)) {
    if (!s.empty() && std::all_of(s.begin(), s.end(), ::isdigit)) v.push_back(atoi(s.c_str()));
  }
  std::sort(v.begin(), v.end());
  return v;
}

int partition_count(const std::string& s) {
  std::string t = trim(s);
  if (t == "SPX") return 1;
  if (t == "DPX") return 2;
  if (t == "TPX") return 3;
  if (t == "QPX") return 4;
  if (t == "CPX") return 8;
  if (t.size() == 4 && t.compare(0, 3, "NPS") == 0 && isdigit((unsigned char)t[3])) return t[3] - '0';
  return 0;
}

std::string uuid_from_unique(uint64_t uid) {
  char b[40];
  snprintf(b, sizeof b, "GPU-%016llx", (unsigned long long)uid);
  return b;
}

std::string gfx_name(int v) {
  if (v <= 0) return "";
  int major = v / 10000, minor = (v / 100) % 100, step = v % 100;
  char b[24];
  snprintf(b, sizeof b, "gfx%d%d%x", major, minor, step);
  return b;
}

std::string bdf_string(uint64_t domain, uint64_t location_id) {
  char b[24];
  snprintf(b, sizeof b, "%04llx:%02llx:%02llx.%llx", (unsigned long long)domain,
           (unsigned long long)((location_id >> 8) & 0xff), (unsigned long long)((location_id >> 3) & 0x1f),
           (unsigned long long)(location_id & 0x7));
  return b;
}

struct LinkMatrix {
  int n = 0;
  std::vector<gs_link_t> m;
  void resize(int k) {
    n = k;
    m.assign((size_t)k * k, gs_link_t{});
    for (int i = 0; i < k; ++i) m[(size_t)i * k + i] = gs_link_t{GS_LINK_SELF, 0, 0, 0, 0};
  }
  gs_link_t& at(int i, int j) { return m[(size_t)i * n + j]; }
  const gs_link_t& at(int i, int j) const { return m[(size_t)i * n + j]; }
};

// Functional probe: amdgpu's gpu_metrics table, which the driver reads from the SMU and refuses
// (EPERM/EBUSY) while the GPU is in reset or not initialised. 1 = answered, 0 = the file is there
// and the read failed (enumerated but not functional), -1 = no such file (unknown here).
int probe_gpu_metrics(const std::string& root, int render_minor) {
  if (render_minor < 0) return -1;
  std::string path = root + "/sys/class/drm/renderD" + std::to_string(render_minor) + "/device/gpu_metrics";
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno == ENOENT ? -1 : 0;
  unsigned char hdr[64];
  ssize_t n = read(fd, hdr, sizeof hdr);
  close(fd);
  // metrics_table_header: structure_size (u16), format_revision (u8), content_revision (u8)
  return n >= 4 && (hdr[0] | hdr[1]) != 0 && hdr[2] != 0 ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// backends
// ---------------------------------------------------------------------------------------
class Backend {
 public:
  // is the device working, beyond being enumerated (see probe_gpu_metrics)
  virtual int probe(const gs_device_t& d) { return probe_gpu_metrics("", d.render_minor); }
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  virtual bool enumerate(std::vector<gs_device_t>* devs, LinkMatrix* links, int* inaccessible) = 0;
  virtual bool events_start(const std::vector<gs_device_t>&) { return true; }
  virtual int wait_event(int timeout_ms, gs_event_t*) {
    if (timeout_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(timeout_ms));
    return 0;
  }
  virtual int inject(const std::string& cmd) {
    set_err(std::string("fault injection unsupported on backend ") + name() + ": " + cmd);
    return -1;
  }
  gs_health_status_t status() const {
    std::lock_guard<std::mutex> lk(st_mu_);
    return st_;
  }

 protected:
  // ECC bookkeeping of one enumeration pass: begin, one note per device, end.
  void ecc_begin() { ecc_ok_ = ecc_fail_ = 0; }
  void ecc_note(int rc) {
    if (rc == 0) {
      ++ecc_ok_;
    } else {
      ++ecc_fail_;
      ecc_rc_ = rc;
    }
  }
  void ecc_end(bool api) {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.ecc_api = api ? 1 : 0;
    st_.ecc_reads_ok = ecc_ok_;
    st_.ecc_reads_failed = ecc_fail_;
    st_.ecc_last_status = ecc_rc_;
    ++st_.refreshes;
  }
  void events_note(bool api, int armed, int last_rc) {
    std::lock_guard<std::mutex> lk(st_mu_);
    st_.events_api = api ? 1 : 0;
    st_.events_armed = armed;
    st_.events_last_status = last_rc;
  }

 private:
  mutable std::mutex st_mu_;
  gs_health_status_t st_{};
  int ecc_ok_ = 0, ecc_fail_ = 0, ecc_rc_ = 0;
};

// ---- sysfs -------------------------------------------------------------------------------
class SysfsBackend : public Backend {
 public:
  explicit SysfsBackend(std::string root) : root_(std::move(root)) {}
  const char* name() const override { return "sysfs"; }
  int probe(const gs_device_t& d) override { return probe_gpu_metrics(root_, d.render_minor); }

  // Enriches a device whose render minor is known from amdgpu's DRM sysfs.
  // Returns true when the RAS (ECC) counters were read.
  bool enrich_from_drm(gs_device_t* d) const {
    if (d->render_minor < 0) return false;
    std::string dev = root_ + "/sys/class/drm/renderD" + std::to_string(d->render_minor) + "/device/";
    std::string v = read_trim(dev + "mem_info_vram_total");
    if (!v.empty()) d->vram_total = to_u64(v);
    v = read_trim(dev + "mem_info_vram_used");
    if (!v.empty()) d->vram_used = to_u64(v);
    v = read_trim(dev + "product_name");
    if (!v.empty()) copy_str(d->name, v);
    v = read_trim(dev + "numa_node");
    if (!v.empty()) d->numa_node = (int32_t)to_i64(v, -1);
    v = read_trim(dev + "current_compute_partition");
    if (!v.empty()) d->compute_partition = partition_count(v);
    v = read_trim(dev + "current_memory_partition");
    if (!v.empty()) d->memory_partition = partition_count(v);
    std::string ras;
    if (read_file(dev + "ras/umc_err_count", &ras)) {
      auto m = parse_props([&] {  // "ue: N\nce: M" -> "ue N"
        std::string t = ras;
        std::replace(t.begin(), t.end(), ':', ' ');
        return t;
      }());
      d->ecc_ue = to_u64(m["ue"]);
      d->ecc_ce = to_u64(m["ce"]);
      return true;
    }
    return false;
  }

  bool enumerate(std::vector<gs_device_t>* devs, LinkMatrix* links, int* inaccessible) override {
    std::string base = root_ + "/sys/class/kfd/kfd/topology/nodes";
    std::vector<int> nodes = numeric_entries(base);
    if (nodes.empty()) {
      set_err("no KFD topology at " + base);
      return false;
    }
    devs->clear();
    *inaccessible = 0;
    ecc_begin();
    std::map<int, int> node_to_idx;
    std::vector<int> gpu_nodes;
    for (int n : nodes) {
      std::string props;
      int err = 0;
      std::string nd = base + "/" + std::to_string(n);
      if (!read_file(nd + "/properties", &props, &err)) {
        // A restricted container sees the node directory but may not read it (EPERM):
        // that is a GPU we are not allowed to manage, not an error.
        ++*inaccessible;
        continue;
      }
      auto p = parse_props(props);
      if (to_u64(p["simd_count"]) == 0) continue;  // CPU node
      gs_device_t d{};
      d.index = (int32_t)devs->size();
      d.kfd_node = n;
      d.render_minor = (int32_t)to_i64(p["drm_render_minor"], -1);
      d.numa_node = -1;
      d.health = GS_HEALTHY;
      d.unique_id = to_u64(p["unique_id"]);
      d.hive_id = to_u64(p["hive_id"]);
      d.num_xcc = (int32_t)to_u64(p["num_xcc"], 1);
      uint64_t simd_per_cu = to_u64(p["simd_per_cu"], 4);
      d.num_cu = (int32_t)(simd_per_cu ? to_u64(p["simd_count"]) / simd_per_cu : 0);
      d.gfx_version = (int32_t)to_u64(p["gfx_target_version"]);
      copy_str(d.gfx, gfx_name(d.gfx_version));
      copy_str(d.uuid, uuid_from_unique(d.unique_id));
      copy_str(d.bdf, bdf_string(to_u64(p["domain"]), to_u64(p["location_id"])));
      // VRAM fallback from KFD mem banks (heap_type 1 = FB public, 2 = FB private).
      uint64_t banks = 0;
      for (int b : numeric_entries(nd + "/mem_banks")) {
        std::string bp;
        if (read_file(nd + "/mem_banks/" + std::to_string(b) + "/properties", &bp)) {
          auto bm = parse_props(bp);
          uint64_t ht = to_u64(bm["heap_type"]);
          if (ht == 1 || ht == 2) banks += to_u64(bm["size_in_bytes"]);
        }
      }
      d.vram_total = banks;
      ecc_note(enrich_from_drm(&d) ? 0 : -1);
      if (d.name[0] == 0) copy_str(d.name, "AMD Instinct GPU");
      node_to_idx[n] = d.index;
      gpu_nodes.push_back(n);
      devs->push_back(d);
    }
    links->resize((int)devs->size());
    for (size_t i = 0; i < gpu_nodes.size(); ++i) {
      std::string nd = base + "/" + std::to_string(gpu_nodes[i]);
      for (const char* kind : {"io_links", "p2p_links"}) {
        for (int l : numeric_entries(nd + "/" + kind)) {
          std::string lp;
          if (!read_file(nd + "/" + kind + "/" + std::to_string(l) + "/properties", &lp)) continue;
          auto m = parse_props(lp);
          int to = (int)to_i64(m["node_to"], -1);
          auto it = node_to_idx.find(to);
          if (it == node_to_idx.end()) continue;
          uint64_t t = to_u64(m["type"]);
          gs_link_t& L = links->at((int)i, it->second);
          if (L.type == GS_LINK_XGMI) continue;  // io_links xGMI wins over p2p entries
          L.type = (t == 11) ? GS_LINK_XGMI : GS_LINK_PCIE;
          L.hops = (t == 11 && std::string(kind) == "io_links") ? 1 : 2;
          L.weight = (int32_t)to_u64(m["weight"]);
          L.max_bandwidth_mbps = to_u64(m["max_bandwidth"]);
        }
      }
    }
    // Any remaining unlinked pair of accessible GPUs talks over PCIe through the host.
    for (int i = 0; i < links->n; ++i)
      for (int j = 0; j < links->n; ++j)
        if (i != j && links->at(i, j).type == GS_LINK_NONE) links->at(i, j) = gs_link_t{GS_LINK_PCIE, 3, 40, 0, 0};
    ecc_end(true);
    return true;
  }

 private:
  std::string root_;
};

// ---- rocm_smi (dlopen) -------------------------------------------------------------------
// Types mirrored from rocm_smi.h (ROCm 7.2: rocm_smi.h:319-351, :697-703, :1249-1252).
struct rsmi_evt_data {
  uint32_t dv_ind;
  int32_t event;
  char message[96];
};
struct rsmi_err_count {
  uint64_t correctable, uncorrectable;
};

class RocmSmiBackend : public Backend {
 public:
  const char* name() const override { return "rocm_smi"; }
  ~RocmSmiBackend() override {
    if (lib_) {
      if (events_on_ && ev_stop_)
        for (uint32_t i = 0; i < n_; ++i) ev_stop_(i);
      if (shut_) shut_();
      dlclose(lib_);
    }
  }

  bool load() {
    const char* names[] = {"librocm_smi64.so.1", "librocm_smi64.so", "/opt/rocm/lib/librocm_smi64.so.1"};
    for (auto nm : names)
      if ((lib_ = dlopen(nm, RTLD_NOW | RTLD_LOCAL))) break;
    if (!lib_) {
      set_err(std::string("dlopen librocm_smi64 failed: ") + dlerror());
      return false;
    }
#define SYM(var, nm)                                                   \
  var = reinterpret_cast<decltype(var)>(dlsym(lib_, nm));              \
  if (!var) {                                                          \
    set_err(std::string("librocm_smi64 lacks ") + nm);                 \
    return false;                                                      \
  }
    SYM(init_, "rsmi_init");
    SYM(shut_, "rsmi_shut_down");
    SYM(num_, "rsmi_num_monitor_devices");
    SYM(uid_, "rsmi_dev_unique_id_get");
    SYM(memtot_, "rsmi_dev_memory_total_get");
    SYM(memuse_, "rsmi_dev_memory_usage_get");
    SYM(pci_, "rsmi_dev_pci_id_get");
    SYM(numa_, "rsmi_topo_numa_affinity_get");
    SYM(linktype_, "rsmi_topo_get_link_type");
    SYM(linkw_, "rsmi_topo_get_link_weight");
#undef SYM
    // optional symbols
    node_ = reinterpret_cast<decltype(node_)>(dlsym(lib_, "rsmi_dev_node_id_get"));
    hive_ = reinterpret_cast<decltype(hive_)>(dlsym(lib_, "rsmi_dev_xgmi_hive_id_get"));
    ecc_ = reinterpret_cast<decltype(ecc_)>(dlsym(lib_, "rsmi_dev_ecc_count_get"));
    bw_ = reinterpret_cast<decltype(bw_)>(dlsym(lib_, "rsmi_minmax_bandwidth_get"));
    ev_init_ = reinterpret_cast<decltype(ev_init_)>(dlsym(lib_, "rsmi_event_notification_init"));
    ev_mask_ = reinterpret_cast<decltype(ev_mask_)>(dlsym(lib_, "rsmi_event_notification_mask_set"));
    ev_get_ = reinterpret_cast<decltype(ev_get_)>(dlsym(lib_, "rsmi_event_notification_get"));
    ev_stop_ = reinterpret_cast<decltype(ev_stop_)>(dlsym(lib_, "rsmi_event_notification_stop"));
    int rc = init_(0);
    if (rc != 0) {
      set_err("rsmi_init failed with status " + std::to_string(rc));
      return false;
    }
    return true;
  }

  bool enumerate(std::vector<gs_device_t>* devs, LinkMatrix* links, int* inaccessible) override {
    uint32_t n = 0;
    if (num_(&n) != 0) {
      set_err("rsmi_num_monitor_devices failed");
      return false;
    }
    n_ = n;
    devs->clear();
    *inaccessible = 0;
    ecc_begin();
    SysfsBackend sysfs("");
    // sysfs view for render minors / partitions / names keyed by unique id.
    std::vector<gs_device_t> sdevs;
    LinkMatrix slinks;
    int sinacc = 0;
    std::map<uint64_t, gs_device_t> by_uid;
    if (sysfs.enumerate(&sdevs, &slinks, &sinacc)) {
      for (auto& d : sdevs) by_uid[d.unique_id] = d;
      *inaccessible = sinacc;
    }
    for (uint32_t i = 0; i < n; ++i) {
      gs_device_t d{};
      d.index = (int32_t)i;
      d.kfd_node = -1;
      d.render_minor = -1;
      d.numa_node = -1;
      d.health = GS_HEALTHY;
      uid_(i, &d.unique_id);
      auto it = by_uid.find(d.unique_id);
      if (it != by_uid.end()) {
        d = it->second;  // take sysfs detail, then override with SMI values
        d.index = (int32_t)i;
      } else {
        copy_str(d.uuid, uuid_from_unique(d.unique_id));
        copy_str(d.name, "AMD Instinct GPU");
      }
      uint64_t v = 0;
      if (memtot_(i, 0 /*RSMI_MEM_TYPE_VRAM*/, &v) == 0) d.vram_total = v;
      if (memuse_(i, 0, &v) == 0) d.vram_used = v;
      uint64_t bdf = 0;
      if (pci_(i, &bdf) == 0) {
        // rsmi BDFID: domain<<32 | bus<<8 | dev<<3 | fn
        copy_str(d.bdf, bdf_string(bdf >> 32, bdf & 0xffff));
      }
      int32_t numa = -1;
      if (numa_(i, &numa) == 0) d.numa_node = numa;
      uint32_t node = 0;
      if (node_ && node_(i, &node) == 0) d.kfd_node = (int32_t)node;
      uint64_t hive = 0;
      if (hive_ && hive_(i, &hive) == 0) d.hive_id = hive;
      rsmi_err_count ec{};
      // RSMI_GPU_BLOCK_UMC = 0x1 (rocm_smi.h rsmi_gpu_block_t): the HBM memory controllers
      int erc = ecc_ ? ecc_(i, 0x1, &ec) : -1;
      if (ecc_) ecc_note(erc);
      if (erc == 0) {
        d.ecc_ue = ec.uncorrectable;
        d.ecc_ce = ec.correctable;
      }
      devs->push_back(d);
    }
    links->resize((int)n);
    for (uint32_t i = 0; i < n; ++i)
      for (uint32_t j = 0; j < n; ++j) {
        if (i == j) continue;
        uint64_t hops = 0, w = 0, bmin = 0, bmax = 0;
        int32_t t = 0;
        gs_link_t L{GS_LINK_PCIE, 3, 40, 0, 0};
        if (linktype_(i, j, &hops, &t) == 0) {
          L.type = (t == 2) ? GS_LINK_XGMI : GS_LINK_PCIE;  // RSMI_IOLINK_TYPE_XGMI == 2
          L.hops = (int32_t)hops;
        }
        if (linkw_(i, j, &w) == 0) L.weight = (int32_t)w;
        if (bw_ && bw_(i, j, &bmin, &bmax) == 0) L.max_bandwidth_mbps = bmax;
        links->at((int)i, (int)j) = L;
      }
    ecc_end(ecc_ != nullptr);
    return true;
  }

  bool events_start(const std::vector<gs_device_t>& devs) override {
    if (!ev_init_ || !ev_mask_ || !ev_get_) return true;  // polling only
    // VMFAULT(1) THERMAL_THROTTLE(2) GPU_PRE_RESET(3) GPU_POST_RESET(4), rocm_smi.h:319-323
    uint64_t mask = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3);
    int armed = 0, last = 0;
    for (auto& d : devs) {
      int rc = ev_init_((uint32_t)d.index);
      if (rc == 0) rc = ev_mask_((uint32_t)d.index, mask);
      if (rc == 0) ++armed; else last = rc;
    }
    events_on_ = armed > 0;
    events_note(true, armed, last);
    return true;
  }

  int wait_event(int timeout_ms, gs_event_t* ev) override {
    if (!events_on_) return Backend::wait_event(timeout_ms, ev);
    rsmi_evt_data data[1];
    uint32_t num = 1;
    int rc = ev_get_(timeout_ms, &num, data);
    if (rc != 0 || num == 0) return 0;
    ev->index = (int32_t)data[0].dv_ind;
    switch (data[0].event) {
      case 1: ev->kind = GS_EV_VMFAULT; break;
      case 2: ev->kind = GS_EV_THERMAL; break;
      case 3: ev->kind = GS_EV_PRE_RESET; break;
      case 4: ev->kind = GS_EV_POST_RESET; break;
      default: ev->kind = GS_EV_NONE; break;
    }
    copy_str(ev->message, std::string(data[0].message, strnlen(data[0].message, sizeof data[0].message)));
    return 1;
  }

 private:
  void* lib_ = nullptr;
  uint32_t n_ = 0;
  bool events_on_ = false;
  int (*init_)(uint64_t) = nullptr;
  int (*shut_)() = nullptr;
  int (*num_)(uint32_t*) = nullptr;
  int (*uid_)(uint32_t, uint64_t*) = nullptr;
  int (*memtot_)(uint32_t, int, uint64_t*) = nullptr;
  int (*memuse_)(uint32_t, int, uint64_t*) = nullptr;
  int (*pci_)(uint32_t, uint64_t*) = nullptr;
  int (*numa_)(uint32_t, int32_t*) = nullptr;
  int (*linktype_)(uint32_t, uint32_t, uint64_t*, int32_t*) = nullptr;
  int (*linkw_)(uint32_t, uint32_t, uint64_t*) = nullptr;
  int (*node_)(uint32_t, uint32_t*) = nullptr;
  int (*hive_)(uint32_t, uint64_t*) = nullptr;
  int (*ecc_)(uint32_t, int, rsmi_err_count*) = nullptr;
  int (*bw_)(uint32_t, uint32_t, uint64_t*, uint64_t*) = nullptr;
  int (*ev_init_)(uint32_t) = nullptr;
  int (*ev_mask_)(uint32_t, uint64_t) = nullptr;
  int (*ev_get_)(int, uint32_t*, rsmi_evt_data*) = nullptr;
  int (*ev_stop_)(uint32_t) = nullptr;
};

// ---- amdsmi (dlopen) ---------------------------------------------------------------------
// The newer AMD SMI library (libamd_smi, /opt/rocm/include/amd_smi/amdsmi.h). Handle-based:
// sockets -> processors; each GPU processor is matched to its sysfs/KFD view by PCI BDF (render
// minor, KFD node, partitions, name), then SMI values (HBM, NUMA, hive, ECC, links) override.
// Only the types used are mirrored (amdsmi.h, ROCm 7.2: :51, :287, :668-677, :760-773,
// :1029-1030, :1336-1341, :1362-1370, :1570, :2090-2098) so the library still builds without ROCm.
struct amdsmi_xgmi_info {
  uint8_t xgmi_lanes;
  uint64_t xgmi_hive_id;
  uint64_t xgmi_node_id;
  uint32_t index;
  uint32_t reserved[9];
};
struct amdsmi_error_count {
  uint64_t correctable_count, uncorrectable_count, deferred_count, reserved[5];
};
struct amdsmi_evt_data {
  void* processor_handle;
  int32_t event;
  char message[256];
};

class AmdSmiBackend : public Backend {
 public:
  const char* name() const override { return "amdsmi"; }
  ~AmdSmiBackend() override {
    if (lib_) {
      if (events_on_ && ev_stop_)
        for (void* h : handles_) ev_stop_(h);
      if (shut_) shut_();
      dlclose(lib_);
    }
  }

  bool load() {
    const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
    for (auto nm : names)
      if ((lib_ = dlopen(nm, RTLD_NOW | RTLD_LOCAL))) break;
    if (!lib_) {
      set_err(std::string("dlopen libamd_smi failed: ") + dlerror());
      return false;
    }
#define SYM(var, nm)                                                   \
  var = reinterpret_cast<decltype(var)>(dlsym(lib_, nm));              \
  if (!var) {                                                          \
    set_err(std::string("libamd_smi lacks ") + nm);                    \
    return false;                                                      \
  }
    SYM(init_, "amdsmi_init");
    SYM(shut_, "amdsmi_shut_down");
    SYM(sockets_, "amdsmi_get_socket_handles");
    SYM(procs_, "amdsmi_get_processor_handles");
    SYM(ptype_, "amdsmi_get_processor_type");
    SYM(bdf_, "amdsmi_get_gpu_device_bdf");
    SYM(memtot_, "amdsmi_get_gpu_memory_total");
#undef SYM
    memuse_ = reinterpret_cast<decltype(memuse_)>(dlsym(lib_, "amdsmi_get_gpu_memory_usage"));
    numa_ = reinterpret_cast<decltype(numa_)>(dlsym(lib_, "amdsmi_topo_get_numa_node_number"));
    linktype_ = reinterpret_cast<decltype(linktype_)>(dlsym(lib_, "amdsmi_topo_get_link_type"));
    linkw_ = reinterpret_cast<decltype(linkw_)>(dlsym(lib_, "amdsmi_topo_get_link_weight"));
    xgmi_ = reinterpret_cast<decltype(xgmi_)>(dlsym(lib_, "amdsmi_get_xgmi_info"));
    ecc_ = reinterpret_cast<decltype(ecc_)>(dlsym(lib_, "amdsmi_get_gpu_total_ecc_count"));
    cpart_ = reinterpret_cast<decltype(cpart_)>(dlsym(lib_, "amdsmi_get_gpu_compute_partition"));
    mpart_ = reinterpret_cast<decltype(mpart_)>(dlsym(lib_, "amdsmi_get_gpu_memory_partition"));
    ev_init_ = reinterpret_cast<decltype(ev_init_)>(dlsym(lib_, "amdsmi_init_gpu_event_notification"));
    ev_mask_ = reinterpret_cast<decltype(ev_mask_)>(dlsym(lib_, "amdsmi_set_gpu_event_notification_mask"));
    ev_get_ = reinterpret_cast<decltype(ev_get_)>(dlsym(lib_, "amdsmi_get_gpu_event_notification"));
    ev_stop_ = reinterpret_cast<decltype(ev_stop_)>(dlsym(lib_, "amdsmi_stop_gpu_event_notification"));
    int rc = init_(1ull << 1 /*AMDSMI_INIT_AMD_GPUS*/);
    if (rc != 0) {
      set_err("amdsmi_init failed with status " + std::to_string(rc));
      return false;
    }
    return true;
  }

  bool enumerate(std::vector<gs_device_t>* devs, LinkMatrix* links, int* inaccessible) override {
    // processors of every socket, GPUs only
    ecc_begin();
    uint32_t ns = 0;
    if (sockets_(&ns, nullptr) != 0) {
      set_err("amdsmi_get_socket_handles failed");
      return false;
    }
    std::vector<void*> socks(ns);
    if (ns && sockets_(&ns, socks.data()) != 0) {
      set_err("amdsmi_get_socket_handles failed");
      return false;
    }
    std::vector<void*> gpus;
    for (void* sk : socks) {
      uint32_t np = 0;
      if (procs_(sk, &np, nullptr) != 0 || !np) continue;
      std::vector<void*> ps(np);
      if (procs_(sk, &np, ps.data()) != 0) continue;
      for (void* p : ps) {
        int32_t t = 0;
        if (ptype_(p, &t) == 0 && t == 1 /*AMDSMI_PROCESSOR_TYPE_AMD_GPU*/) gpus.push_back(p);
      }
    }
    // sysfs detail keyed by BDF; its order (KFD / HIP ordinal order) decides device indices
    SysfsBackend sysfs("");
    std::vector<gs_device_t> sdevs;
    LinkMatrix slinks;
    int sinacc = 0;
    std::map<std::string, gs_device_t> by_bdf;
    *inaccessible = 0;
    if (sysfs.enumerate(&sdevs, &slinks, &sinacc)) {
      for (auto& d : sdevs) by_bdf[d.bdf] = d;
      *inaccessible = sinacc;
    }
    struct Entry {
      gs_device_t d;
      void* h;
      int order;
    };
    std::vector<Entry> es;
    for (size_t k = 0; k < gpus.size(); ++k) {
      void* h = gpus[k];
      gs_device_t d{};
      d.kfd_node = d.render_minor = d.numa_node = -1;
      d.health = GS_HEALTHY;
      uint64_t b = 0;
      char bdf[32] = {0};
      if (bdf_(h, &b) == 0)
        snprintf(bdf, sizeof bdf, "%04llx:%02llx:%02llx.%llx", (unsigned long long)(b >> 16),
                 (unsigned long long)((b >> 8) & 0xff), (unsigned long long)((b >> 3) & 0x1f),
                 (unsigned long long)(b & 0x7));
      int order = 1000 + (int)k;
      auto it = by_bdf.find(bdf);
      if (it != by_bdf.end()) {
        d = it->second;
        order = it->second.index;
      } else {
        copy_str(d.name, "AMD Instinct GPU");
      }
      copy_str(d.bdf, bdf);
      uint64_t v = 0;
      if (memtot_(h, 0 /*AMDSMI_MEM_TYPE_VRAM*/, &v) == 0) d.vram_total = v;
      if (memuse_ && memuse_(h, 0, &v) == 0) d.vram_used = v;
      uint32_t numa = 0;
      if (numa_ && numa_(h, &numa) == 0) d.numa_node = (int32_t)numa;
      amdsmi_xgmi_info xi{};
      if (xgmi_ && xgmi_(h, &xi) == 0) d.hive_id = xi.xgmi_hive_id;
      amdsmi_error_count ec{};
      int erc = ecc_ ? ecc_(h, &ec) : -1;
      if (ecc_) ecc_note(erc);
      if (erc == 0) {
        d.ecc_ue = ec.uncorrectable_count;
        d.ecc_ce = ec.correctable_count;
      }
      char part[32] = {0};
      if (cpart_ && cpart_(h, part, sizeof part) == 0 && partition_count(part) > 0)
        d.compute_partition = partition_count(part);
      if (mpart_ && mpart_(h, part, sizeof part) == 0 && partition_count(part) > 0)
        d.memory_partition = partition_count(part);
      if (!d.uuid[0]) copy_str(d.uuid, uuid_from_unique(d.unique_id));
      es.push_back({d, h, order});
    }
    std::stable_sort(es.begin(), es.end(), [](const Entry& a, const Entry& b) { return a.order < b.order; });
    ecc_end(ecc_ != nullptr);
    devs->clear();
    handles_.clear();
    for (size_t i = 0; i < es.size(); ++i) {
      es[i].d.index = (int32_t)i;
      devs->push_back(es[i].d);
      handles_.push_back(es[i].h);
    }
    int n = (int)es.size();
    links->resize(n);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        if (i == j) continue;
        gs_link_t L{GS_LINK_PCIE, 3, 40, 0, 0};
        uint64_t hops = 0, w = 0;
        int32_t t = 0;
        if (linktype_ && linktype_(handles_[i], handles_[j], &hops, &t) == 0) {
          L.type = (t == 2 /*AMDSMI_LINK_TYPE_XGMI*/) ? GS_LINK_XGMI : GS_LINK_PCIE;
          L.hops = (int32_t)hops;
        }
        if (linkw_ && linkw_(handles_[i], handles_[j], &w) == 0) L.weight = (int32_t)w;
        if (L.type == GS_LINK_XGMI && i < slinks.n && j < slinks.n)
          L.max_bandwidth_mbps = slinks.at(i, j).max_bandwidth_mbps;
        links->at(i, j) = L;
      }
    return true;
  }

  bool events_start(const std::vector<gs_device_t>&) override {
    if (!ev_init_ || !ev_mask_ || !ev_get_) return true;  // polling only
    uint64_t mask = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3);  // events 1..4, bit = event - 1
    int armed = 0, last = 0;
    for (void* h : handles_) {
      int rc = ev_init_(h);
      if (rc == 0) rc = ev_mask_(h, mask);
      if (rc == 0) ++armed; else last = rc;
    }
    events_on_ = armed > 0;
    events_note(true, armed, last);
    return true;
  }

  int wait_event(int timeout_ms, gs_event_t* ev) override {
    if (!events_on_) return Backend::wait_event(timeout_ms, ev);
    amdsmi_evt_data data[1];
    uint32_t num = 1;
    if (ev_get_(timeout_ms, &num, data) != 0 || num == 0) return 0;
    ev->index = -1;
    for (size_t i = 0; i < handles_.size(); ++i)
      if (handles_[i] == data[0].processor_handle) ev->index = (int32_t)i;
    switch (data[0].event) {
      case 1: ev->kind = GS_EV_VMFAULT; break;
      case 2: ev->kind = GS_EV_THERMAL; break;
      case 3: ev->kind = GS_EV_PRE_RESET; break;
      case 4: ev->kind = GS_EV_POST_RESET; break;
      default: ev->kind = GS_EV_NONE; break;
    }
    copy_str(ev->message, std::string(data[0].message, strnlen(data[0].message, sizeof data[0].message)));
    return 1;
  }

 private:
  void* lib_ = nullptr;
  std::vector<void*> handles_;
  bool events_on_ = false;
  int (*init_)(uint64_t) = nullptr;
  int (*shut_)() = nullptr;
  int (*sockets_)(uint32_t*, void**) = nullptr;
  int (*procs_)(void*, uint32_t*, void**) = nullptr;
  int (*ptype_)(void*, int32_t*) = nullptr;
  int (*bdf_)(void*, uint64_t*) = nullptr;
  int (*memtot_)(void*, int, uint64_t*) = nullptr;
  int (*memuse_)(void*, int, uint64_t*) = nullptr;
  int (*numa_)(void*, uint32_t*) = nullptr;
  int (*linktype_)(void*, void*, uint64_t*, int32_t*) = nullptr;
  int (*linkw_)(void*, void*, uint64_t*) = nullptr;
  int (*xgmi_)(void*, amdsmi_xgmi_info*) = nullptr;
  int (*ecc_)(void*, amdsmi_error_count*) = nullptr;
  int (*cpart_)(void*, char*, uint32_t) = nullptr;
  int (*mpart_)(void*, char*, uint32_t) = nullptr;
  int (*ev_init_)(void*) = nullptr;
  int (*ev_mask_)(void*, uint64_t) = nullptr;
  int (*ev_get_)(int, uint32_t*, amdsmi_evt_data*) = nullptr;
  int (*ev_stop_)(void*) = nullptr;
};

// ---- fake (tests, simulation, fault injection) -------------------------------------------
class FakeBackend : public Backend {
 public:
  const char* name() const override { return "fake"; }
  // "resetting I N": the device stays enumerated but fails the probe on its next N probes
  int probe(const gs_device_t& d) override {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < all_.size(); ++i)
      if (std::strcmp(all_[i].uuid, d.uuid) == 0) {
        auto it = probe_fail_.find((int)i);
        if (it == probe_fail_.end() || it->second <= 0) return 1;
        --it->second;
        return 0;
      }
    return -1;
  }
  bool events_start(const std::vector<gs_device_t>& devs) override {
    events_note(true, (int)devs.size(), 0);  // injected events are always delivered
    return true;
  }

  bool configure(const std::string& spec) {
    // "<N>x<SIZE>[G|M|B]" shorthand, e.g. "8x288G", "2x4G"; otherwise a JSON file path.
    size_t x = spec.find('x');
    if (x != std::string::npos && x > 0 && std::all_of(spec.begin(), spec.begin() + x, ::isdigit)) {
      int n = atoi(spec.substr(0, x).c_str());
      std::string sz = spec.substr(x + 1);
      uint64_t mult = 1;
      if (!sz.empty() && (sz.back() == 'G' || sz.back() == 'g')) mult = 1ull << 30, sz.pop_back();
      else if (!sz.empty() && (sz.back() == 'M' || sz.back() == 'm')) mult = 1ull << 20, sz.pop_back();
      else if (!sz.empty() && (sz.back() == 'B' || sz.back() == 'b')) sz.pop_back();
      double v = atof(sz.c_str());
      if (n <= 0 || n > 64 || v <= 0) {
        set_err("bad fake spec " + spec);
        return false;
      }
      for (int i = 0; i < n; ++i) all_.push_back(make_dev(i, (uint64_t)(v * (double)mult)));
      full_xgmi(n);
      return true;
    }
    std::string text;
    if (!read_file(spec, &text)) {
      set_err("cannot read fake spec file " + spec);
      return false;
    }
    jsonmin::Value root;
    std::string perr;
    if (!jsonmin::parse(text, &root, &perr)) {
      set_err("fake spec JSON: " + perr);
      return false;
    }
    const jsonmin::Value* arr = root.get("devices");
    if (!arr || !arr->is_array()) {
      set_err("fake spec JSON needs a \"devices\" array");
      return false;
    }
    int i = 0;
    for (const auto& jd : arr->arr) {
      gs_device_t d = make_dev(i, (uint64_t)jd.num_or("vram_total", 4.0 * (1ull << 30)));
      if (auto s = jd.get("uuid"); s && s->is_string()) copy_str(d.uuid, s->str);
      if (auto s = jd.get("bdf"); s && s->is_string()) copy_str(d.bdf, s->str);
      if (auto s = jd.get("name"); s && s->is_string()) copy_str(d.name, s->str);
      d.numa_node = (int32_t)jd.num_or("numa_node", d.numa_node);
      d.render_minor = (int32_t)jd.num_or("render_minor", d.render_minor);
      d.hive_id = (uint64_t)jd.num_or("hive_id", (double)d.hive_id);
      d.unique_id = (uint64_t)jd.num_or("unique_id", (double)d.unique_id);
      d.compute_partition = (int32_t)jd.num_or("compute_partition", 1);
      d.memory_partition = (int32_t)jd.num_or("memory_partition", 1);
      d.vram_used = (uint64_t)jd.num_or("vram_used", 0);
      all_.push_back(d);
      ++i;
    }
    int n = (int)all_.size();
    const jsonmin::Value* x2 = root.get("xgmi");
    if (x2 && x2->is_array()) {
      base_links_.resize(n);
      for (int a = 0; a < n && a < (int)x2->arr.size(); ++a)
        for (int b = 0; b < n && b < (int)x2->arr[a].arr.size(); ++b) {
          if (a == b) continue;
          int hops = (int)x2->arr[a].arr[b].num;
          base_links_.at(a, b) = hops == 1 ? gs_link_t{GS_LINK_XGMI, 1, 15, 0, 153600}
                                           : gs_link_t{GS_LINK_PCIE, hops > 0 ? hops : 3, 40, 0, 64000};
        }
    } else if (x2 && x2->is_string() && x2->str == "none") {
      base_links_.resize(n);
      for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b)
          if (a != b) base_links_.at(a, b) = gs_link_t{GS_LINK_PCIE, 3, 40, 0, 64000};
    } else {
      full_xgmi(n);
    }
    return true;
  }

  bool enumerate(std::vector<gs_device_t>* devs, LinkMatrix* links, int* inaccessible) override {
    std::lock_guard<std::mutex> lk(mu_);
    devs->clear();
    *inaccessible = 0;
    std::vector<int> present;
    for (size_t i = 0; i < all_.size(); ++i)
      if (!unplugged_.count((int)i)) present.push_back((int)i);
    ecc_begin();
    for (int k : present) {
      gs_device_t d = all_[k];
      d.index = (int32_t)devs->size();
      devs->push_back(d);
      ecc_note(0);
    }
    ecc_end(true);
    links->resize((int)present.size());
    for (size_t a = 0; a < present.size(); ++a)
      for (size_t b = 0; b < present.size(); ++b) {
        if (a == b) continue;
        gs_link_t L = base_links_.at(present[a], present[b]);
        if (down_.count({std::min(present[a], present[b]), std::max(present[a], present[b])}))
          L = gs_link_t{GS_LINK_PCIE, 3, 40, 0, 64000};
        links->at((int)a, (int)b) = L;
      }
    return true;
  }

  int wait_event(int timeout_ms, gs_event_t* ev) override {
    std::unique_lock<std::mutex> lk(mu_);
    if (!cv_.wait_for(lk, std::chrono::milliseconds(std::max(timeout_ms, 0)), [&] { return !q_.empty(); }))
      return 0;
    *ev = q_.front();
    q_.pop_front();
    return 1;
  }

  int inject(const std::string& cmd) override {
    std::istringstream is(cmd);
    std::string op;
    int a = -1, b = -1;
    is >> op >> a;
    if (op == "linkdown" || op == "linkup" || op == "ecc" || op == "vram" || op == "resetting") is >> b;
    std::lock_guard<std::mutex> lk(mu_);
    if (a < 0 || a >= (int)all_.size()) {
      set_err("inject: bad device index in '" + cmd + "'");
      return -1;
    }
    auto push = [&](int idx, int kind, const std::string& msg) {
      gs_event_t e{};
      e.index = idx;
      e.kind = kind;
      copy_str(e.message, msg);
      q_.push_back(e);
    };
    if (op == "unplug") {
      unplugged_.insert(a);
      push(a, GS_EV_UNPLUG, "device removed");
    } else if (op == "replug") {
      unplugged_.erase(a);
      push(a, GS_EV_REPLUG, "device re-added");
    } else if (op == "reset") {
      push(a, GS_EV_PRE_RESET, "GPU pre-reset");
      push(a, GS_EV_POST_RESET, "GPU post-reset");
    } else if (op == "prereset") {  // a reset whose post-reset event is lost
      push(a, GS_EV_PRE_RESET, "GPU pre-reset");
    } else if (op == "silentreset") {  // a completed reset with no event at all: counters cleared
      all_[a].ecc_ue = 0;
    } else if (op == "resetting") {  // a pre-reset, then the device enumerated but not working for b probes
      probe_fail_[a] = b > 0 ? b : 1;
      push(a, GS_EV_PRE_RESET, "GPU pre-reset");
    } else if (op == "ecc") {
      all_[a].ecc_ue += (uint64_t)(b > 0 ? b : 1);
      push(a, GS_EV_ECC_UE, "uncorrectable ECC error");
    } else if (op == "vram") {  // "vram <idx> <MiB>": the HBM use the backend reports (no event)
      all_[a].vram_used = (uint64_t)(b > 0 ? b : 0) << 20;
    } else if (op == "vmfault") {
      push(a, GS_EV_VMFAULT, "VM fault");
    } else if (op == "thermal") {
      push(a, GS_EV_THERMAL, "thermal throttle");
    } else if (op == "linkdown" || op == "linkup") {
      if (b < 0 || b >= (int)all_.size() || b == a) {
        set_err("inject: bad peer index in '" + cmd + "'");
        return -1;
      }
      auto key = std::make_pair(std::min(a, b), std::max(a, b));
      if (op == "linkdown") down_.insert(key), push(a, GS_EV_LINK_DOWN, "xGMI link down");
      else down_.erase(key), push(a, GS_EV_LINK_UP, "xGMI link up");
    } else {
      set_err("inject: unknown op '" + op + "'");
      return -1;
    }
    cv_.notify_all();
    return 0;
  }

 private:
  gs_device_t make_dev(int i, uint64_t bytes) {
    gs_device_t d{};
    d.index = i;
    d.kfd_node = 2 + i;
    d.render_minor = 128 + 8 * i;
    d.numa_node = i < 4 ? 0 : 1;
    d.health = GS_HEALTHY;
    d.compute_partition = 1;
    d.memory_partition = 1;
    d.num_xcc = 8;
    d.num_cu = 256;
    d.gfx_version = 90500;
    d.unique_id = 0xfa6e000000000000ull + (uint64_t)i;
    d.hive_id = 0x5ca1ab1e00000001ull;
    d.vram_total = bytes;
    copy_str(d.uuid, uuid_from_unique(d.unique_id));
    char bdf[24];
    snprintf(bdf, sizeof bdf, "0000:%02x:00.0", 0x05 + 0x10 * i);
    copy_str(d.bdf, bdf);
    copy_str(d.name, "AMD Instinct MI355X (fake)");
    copy_str(d.gfx, "gfx950");
    return d;
  }
  void full_xgmi(int n) {
    base_links_.resize(n);
    for (int a = 0; a < n; ++a)
      for (int b = 0; b < n; ++b)
        if (a != b) base_links_.at(a, b) = gs_link_t{GS_LINK_XGMI, 1, 15, 0, 153600};
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<gs_device_t> all_;
  LinkMatrix base_links_;
  std::set<int> unplugged_;
  std::map<int, int> probe_fail_;  // device -> probes still to fail ("resetting")
  std::set<std::pair<int, int>> down_;
  std::deque<gs_event_t> q_;
};

}  // namespace

struct gs_handle {
  std::unique_ptr<Backend> be;
  std::mutex mu;
  std::vector<gs_device_t> devs;
  LinkMatrix links;
  int inaccessible = 0;
  std::string backend_name;
};

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }
const char* gs_last_error(void) { return g_err.c_str(); }
const char* gs_backend_name(const gs_handle* h) { return h ? h->backend_name.c_str() : ""; }

int gs_refresh(gs_handle* h) {
  if (!h) return -1;
  std::vector<gs_device_t> devs;
  LinkMatrix links;
  int inacc = 0;
  if (!h->be->enumerate(&devs, &links, &inacc)) return -1;
  std::lock_guard<std::mutex> lk(h->mu);
  h->devs.swap(devs);
  h->links = links;
  h->inaccessible = inacc;
  return (int)h->devs.size();
}

int gs_open(const char* spec_c, gs_handle** out) {
  if (!out) return -1;
  *out = nullptr;
  std::string spec = spec_c ? spec_c : "auto";
  std::unique_ptr<Backend> be;
  std::string nm;
  if (spec.compare(0, 5, "fake:") == 0) {
    auto f = std::make_unique<FakeBackend>();
    if (!f->configure(spec.substr(5))) return -1;
    be = std::move(f);
    nm = "fake";
  } else if (spec == "sysfs" || spec.compare(0, 6, "sysfs:") == 0) {
    be = std::make_unique<SysfsBackend>(spec.size() > 6 ? spec.substr(6) : "");
    nm = "sysfs";
  } else if (spec == "amdsmi") {
    auto a = std::make_unique<AmdSmiBackend>();
    if (!a->load()) return -1;
    be = std::move(a);
    nm = "amdsmi";
  } else if (spec == "rocm_smi" || spec == "auto") {
    auto r = std::make_unique<RocmSmiBackend>();
    if (r->load()) {
      be = std::move(r);
      nm = "rocm_smi";
    } else if (spec == "auto") {
      be = std::make_unique<SysfsBackend>("");
      nm = "sysfs";
    } else {
      return -1;
    }
  } else {
    set_err("unknown backend spec '" + spec + "'");
    return -1;
  }
  auto h = std::make_unique<gs_handle>();
  h->be = std::move(be);
  h->backend_name = nm;
  if (gs_refresh(h.get()) < 0) {
    if (spec == "auto" && nm == "rocm_smi") {  // rocm_smi loaded but failed: fall back
      h->be = std::make_unique<SysfsBackend>("");
      h->backend_name = "sysfs";
      if (gs_refresh(h.get()) < 0) return -1;
    } else {
      return -1;
    }
  }
  if (spec == "auto" && h->backend_name == "rocm_smi" && h->devs.empty()) {
    h->be = std::make_unique<SysfsBackend>("");
    h->backend_name = "sysfs";
    if (gs_refresh(h.get()) < 0) return -1;
  }
  *out = h.release();
  return 0;
}

void gs_close(gs_handle* h) { delete h; }

int gs_device_count(const gs_handle* h) {
  if (!h) return -1;
  std::lock_guard<std::mutex> lk(const_cast<gs_handle*>(h)->mu);
  return (int)h->devs.size();
}

int gs_inaccessible_count(const gs_handle* h) { return h ? h->inaccessible : -1; }

int gs_get_device(const gs_handle* h, int i, gs_device_t* out) {
  if (!h || !out) return -1;
  std::lock_guard<std::mutex> lk(const_cast<gs_handle*>(h)->mu);
  if (i < 0 || i >= (int)h->devs.size()) {
    set_err("device index out of range");
    return -1;
  }
  *out = h->devs[(size_t)i];
  return 0;
}

int gs_get_link(const gs_handle* h, int i, int j, gs_link_t* out) {
  if (!h || !out) return -1;
  std::lock_guard<std::mutex> lk(const_cast<gs_handle*>(h)->mu);
  if (i < 0 || j < 0 || i >= h->links.n || j >= h->links.n) {
    set_err("link index out of range");
    return -1;
  }
  *out = h->links.at(i, j);
  return 0;
}

int gs_events_start(gs_handle* h) {
  if (!h) return -1;
  std::vector<gs_device_t> devs;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    devs = h->devs;
  }
  return h->be->events_start(devs) ? 0 : -1;
}

int gs_wait_event(gs_handle* h, int timeout_ms, gs_event_t* ev) {
  if (!h || !ev) return -1;
  *ev = gs_event_t{};
  return h->be->wait_event(timeout_ms, ev);
}

int gs_health_status(const gs_handle* h, gs_health_status_t* out) {
  if (!h || !out) return -1;
  *out = h->be->status();
  return 0;
}

int gs_inject(gs_handle* h, const char* cmd) {
  if (!h || !cmd) return -1;
  return h->be->inject(cmd);
}

int gs_probe(gs_handle* h, int i) {
  if (!h) return -1;
  gs_device_t d;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (i < 0 || i >= (int)h->devs.size()) {
      set_err("device index out of range");
      return -2;
    }
    d = h->devs[(size_t)i];
  }
  return h->be->probe(d);
}

int gs_to_json(const gs_handle* h, char* buf, size_t len) {
  if (!h) return -1;
  std::lock_guard<std::mutex> lk(const_cast<gs_handle*>(h)->mu);
  std::ostringstream o;
  o << "{\"backend\":\"" << h->backend_name << "\",\"inaccessible\":" << h->inaccessible << ",\"devices\":[";
  for (size_t i = 0; i < h->devs.size(); ++i) {
    const gs_device_t& d = h->devs[i];
    if (i) o << ",";
    o << "{\"index\":" << d.index << ",\"uuid\":\"" << d.uuid << "\",\"bdf\":\"" << d.bdf << "\",\"name\":\""
      << jsonmin::escape(d.name) << "\",\"gfx\":\"" << d.gfx << "\",\"vram_total\":" << d.vram_total
      << ",\"vram_used\":" << d.vram_used << ",\"numa_node\":" << d.numa_node << ",\"render_minor\":"
      << d.render_minor << ",\"kfd_node\":" << d.kfd_node << ",\"unique_id\":" << d.unique_id
      << ",\"hive_id\":" << d.hive_id << ",\"num_xcc\":" << d.num_xcc << ",\"num_cu\":" << d.num_cu
      << ",\"compute_partition\":" << d.compute_partition << ",\"memory_partition\":" << d.memory_partition
      << ",\"ecc_ue\":" << d.ecc_ue << ",\"ecc_ce\":" << d.ecc_ce << ",\"health\":" << d.health << "}";
  }
  o << "],\"links\":[";
  for (int i = 0; i < h->links.n; ++i) {
    if (i) o << ",";
    o << "[";
    for (int j = 0; j < h->links.n; ++j) {
      const gs_link_t& L = h->links.at(i, j);
      if (j) o << ",";
      o << "{\"type\":" << L.type << ",\"hops\":" << L.hops << ",\"weight\":" << L.weight
        << ",\"max_bw_mbps\":" << L.max_bandwidth_mbps << "}";
    }
    o << "]";
  }
  o << "]}";
  std::string s = o.str();
  if (buf && len) {
    size_t n = std::min(s.size(), len - 1);
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)s.size();
}

}  // extern "C"
