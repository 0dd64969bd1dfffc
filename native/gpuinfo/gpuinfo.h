// libgpushare_gpuinfo — MI355X device discovery, topology and health for the gpushare plugin.
//
// Replaces the reference's NVML binding (go-nvml via cgo: pkg/gpu/nvidia/nvidia.go:17-86,
// gpumanager.go:36-41) and its dead XID watcher (nvidia.go:97-153) with an AMD-native C ABI:
//   * "amdsmi"    — libamd_smi (dlopen'ed at runtime), matched to sysfs by PCI BDF;
//   * "rocm_smi"  — librocm_smi64 (dlopen'ed at runtime, so the library builds and loads on
//                    hosts without ROCm), enriched from amdgpu/KFD sysfs;
//   * "sysfs[:<root>]" — /sys/class/kfd topology + /sys/class/drm (root prefix for tests);
//   * "fake:<N>x<SIZE>" or "fake:<file.json>" — synthetic devices with fault injection;
//   * "auto"     — rocm_smi if it initialises and sees a GPU, else sysfs.
// The struct layouts below are mirrored by ctypes in device/smi.py; keep them in sync.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 2

enum gs_health { GS_HEALTHY = 0, GS_UNHEALTHY = 1, GS_MISSING = 2 };
enum gs_link_type { GS_LINK_NONE = 0, GS_LINK_PCIE = 1, GS_LINK_XGMI = 2, GS_LINK_SELF = 3 };
enum gs_event_kind {
  GS_EV_NONE = 0, GS_EV_VMFAULT = 1, GS_EV_THERMAL = 2, GS_EV_PRE_RESET = 3, GS_EV_POST_RESET = 4,
  GS_EV_UNPLUG = 10, GS_EV_REPLUG = 11, GS_EV_ECC_UE = 12, GS_EV_LINK_DOWN = 13, GS_EV_LINK_UP = 14,
};

typedef struct gs_device {
  int32_t index;              // position in enumeration order (HIP ordinal order)
  int32_t kfd_node;           // /sys/class/kfd/kfd/topology/nodes/<n>, -1 unknown
  int32_t render_minor;       // /dev/dri/renderD<minor>, -1 unknown
  int32_t numa_node;          // -1 unknown
  int32_t health;             // gs_health
  int32_t compute_partition;  // partitions per device: 1 SPX, 2 DPX, 4 QPX, 8 CPX; 0 unknown
  int32_t memory_partition;   // NPS1/2/4/8 -> 1/2/4/8; 0 unknown
  int32_t num_xcc;
  int32_t num_cu;
  int32_t gfx_version;        // e.g. 90500 for gfx950
  uint64_t unique_id;
  uint64_t hive_id;
  uint64_t vram_total;        // bytes
  uint64_t vram_used;         // bytes
  uint64_t ecc_ue;            // accumulated uncorrectable errors
  uint64_t ecc_ce;            // accumulated correctable errors
  char uuid[40];              // "GPU-<16 hex>" (ROCR_VISIBLE_DEVICES form)
  char bdf[16];               // "0000:0a:00.0"
  char name[64];              // product name
  char gfx[16];               // "gfx950"
} gs_device_t;

typedef struct gs_link {
  int32_t type;               // gs_link_type
  int32_t hops;
  int32_t weight;
  int32_t reserved;
  uint64_t max_bandwidth_mbps;
} gs_link_t;

typedef struct gs_event {
  int32_t index;              // device index, -1 = all devices
  int32_t kind;               // gs_event_kind
  char message[96];
} gs_event_t;

// What the health path actually has on this backend (so a test on hardware can assert the
// event stream was armed and the ECC counters were read, instead of "no event arrived").
typedef struct gs_health_status {
  int32_t events_api;          // 1: an event-notification API was resolved (rocm_smi / amdsmi)
  int32_t events_armed;        // devices whose notification init + mask succeeded
  int32_t events_last_status;  // last non-zero status from init/mask (0 = none)
  int32_t ecc_api;             // 1: an ECC counter API (or sysfs RAS file) is available
  int32_t ecc_reads_ok;        // devices whose ECC counters were read at the last refresh
  int32_t ecc_reads_failed;    // devices whose ECC read failed at the last refresh
  int32_t ecc_last_status;     // last non-zero status from the ECC read (0 = none)
  int32_t refreshes;           // successful enumerations so far
} gs_health_status_t;

typedef struct gs_handle gs_handle;

int gs_abi_version(void);
// Opens a backend (see header comment). Returns 0 on success; on failure *out is NULL and
// gs_last_error() describes why.
int gs_open(const char* spec, gs_handle** out);
void gs_close(gs_handle* h);
const char* gs_backend_name(const gs_handle* h);
const char* gs_last_error(void);
// Re-enumerates devices (hot-unplug/replug detection, used/ECC counters). Returns count.
int gs_refresh(gs_handle* h);
int gs_device_count(const gs_handle* h);
// GPU nodes present in the topology but not accessible to this process (EPERM in a
// restricted container): they are reported, not silently dropped.
int gs_inaccessible_count(const gs_handle* h);
int gs_get_device(const gs_handle* h, int i, gs_device_t* out);
int gs_get_link(const gs_handle* h, int i, int j, gs_link_t* out);
// Starts hardware event delivery (rocm_smi event notification); harmless elsewhere.
int gs_events_start(gs_handle* h);
// Waits up to timeout_ms for one event. Returns 1 and fills *ev, 0 on timeout, <0 on error.
int gs_wait_event(gs_handle* h, int timeout_ms, gs_event_t* ev);
// Fills *out with the backend's health-path status (see gs_health_status_t).
int gs_health_status(const gs_handle* h, gs_health_status_t* out);
// Fault injection (fake backend only): "unplug I", "replug I", "reset I", "ecc I N",
// "vmfault I", "linkdown I J", "linkup I J", "thermal I", "prereset I", "silentreset I",
// "resetting I N" (a pre-reset, then enumerated but failing gs_probe N times).
int gs_inject(gs_handle* h, const char* cmd);
// Functional probe of device i beyond enumeration (amdgpu gpu_metrics, which the driver refuses
// while the GPU is in reset): 1 working, 0 enumerated but not working, -1 unknown, -2 bad index.
int gs_probe(gs_handle* h, int i);
// Writes a JSON document describing all devices and the link matrix. Returns the number of
// bytes needed (excluding NUL); writes at most len bytes.
int gs_to_json(const gs_handle* h, char* buf, size_t len);

#ifdef __cplusplus
}
#endif
