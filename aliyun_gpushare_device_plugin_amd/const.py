"""Wire contract shared with the kubelet, the gpushare-scheduler-extender and workloads.

Every name here is part of the compatibility surface of the reference plugin and must not
change spelling (reference: ``pkg/gpu/nvidia/const.go:10-36``, ``cmd/inspect/main.go:13-26``,
``device-plugin-ds.yaml:17,23-24``). AMD-specific additions live at the bottom and are
clearly namespaced so that an extender unaware of them keeps working.
"""
from __future__ import annotations

import os

# --- extended resources (const.go:11-12) -------------------------------------------------
RESOURCE_NAME = "aliyun.com/gpu-mem"          # device-plugin managed: Σ GPUs × units/GPU
RESOURCE_COUNT = "aliyun.com/gpu-count"       # node-status patched: number of physical GPUs

# --- kubelet device-plugin API v1beta1 (k8s.io/kubelet v0.28, go.mod:14) ------------------
API_VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET_NAME = "kubelet.sock"
PLUGIN_SOCKET_NAME = "aliyungpushare.sock"    # const.go:13 (serverSock basename)
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

# Fake device id "<UUID>-_-<j>" (nvidia.go:23-29)
FAKE_ID_SEP = "-_-"

# --- pod annotations written by the extender / plugin (const.go:25-31) --------------------
ENV_RESOURCE_INDEX = "ALIYUN_COM_GPU_MEM_IDX"
ENV_RESOURCE_BY_POD = "ALIYUN_COM_GPU_MEM_POD"
ENV_RESOURCE_BY_CONTAINER = "ALIYUN_COM_GPU_MEM_CONTAINER"
ENV_RESOURCE_BY_DEV = "ALIYUN_COM_GPU_MEM_DEV"
ENV_ASSIGNED_FLAG = "ALIYUN_COM_GPU_MEM_ASSIGNED"
ENV_RESOURCE_ASSUME_TIME = "ALIYUN_COM_GPU_MEM_ASSUME_TIME"
ENV_RESOURCE_ASSIGN_TIME = "ALIYUN_COM_GPU_MEM_ASSIGN_TIME"
# newer extender: {"<containerIdx>": {"<gpuIdx>": mem}} (cmd/inspect/main.go:25)
GPUSHARE_ALLOCATION_FLAG = "scheduler.framework.gpushare.allocation"

# --- node label / container env (const.go:32, allocate.go:125-127) -----------------------
NODE_LABEL_DISABLE_CGPU = "cgpu.disable.isolation"
ENV_CGPU_DISABLE = "CGPU_DISABLE"
NODE_SELECTOR_LABEL = ("gpushare", "true")                 # device-plugin-ds.yaml:23-24
PLUGIN_COMPONENT_LABEL = ("component", "gpushare-device-plugin")  # device-plugin-ds.yaml:17

# --- optimistic lock message (const.go:15) -----------------------------------------------
OPTIMISTIC_LOCK_ERROR_MSG = ("the object has been modified; please apply your changes to "
                             "the latest version and try again")

# --- memory units (const.go:34-35) -------------------------------------------------------
GIB = "GiB"
MIB = "MiB"
UNIT_BYTES = {GIB: 1 << 30, MIB: 1 << 20}

# --- AMD-native additions (no reference counterpart) -------------------------------------
# Device nodes injected into every allocated container instead of an NVIDIA runtime hook.
KFD_DEVICE = "/dev/kfd"
DRI_RENDER_FMT = "/dev/dri/renderD{minor}"
# HIP quota shim: host path of the .so is mounted at this container path and preloaded.
SHIM_CONTAINER_DIR = "/usr/local/gpushare"
SHIM_LIB_NAME = "libgpushare_hipquota.so"
ENV_LD_PRELOAD = "LD_PRELOAD"
ENV_SHIM_LEDGER = "GPUSHARE_LEDGER"          # shm ledger name shared by a container's processes
ENV_SHIM_QUOTA_BYTES = "GPUSHARE_QUOTA_BYTES"  # explicit override (tests / debugging)
ENV_SHIM_GRANULE = "GPUSHARE_ALLOC_GRANULE"    # allocation rounding granule override
ENV_SHIM_LOG = "GPUSHARE_SHIM_LOG"
ENV_SHIM_LEDGER_DIR = "GPUSHARE_LEDGER_DIR"    # file-backed ledgers in a host-mounted directory
LEDGER_CONTAINER_DIR = "/run/gpushare/ledger"
# per-GPU HBM broker (native/hbmbroker): the socket directory mounted into shared containers,
# the GPU's socket and the pod's grant token
ENV_HBM_BROKER = "GPUSHARE_HBM_BROKER"
ENV_HBM_TOKEN = "GPUSHARE_HBM_TOKEN"
HBM_BROKER_CONTAINER_DIR = "/run/gpushare/hbm"
# kernel arguments in host memory for a pod on broker memory: with the runtime's default (copied
# into device memory) a hipGraph decode next to a neighbour on broker memory kept 9 % of its solo
# rate, 22 % with this, and solo decode is not slower (profiles/r6/colocate_llama3_8b_x2_broker.json)
ENV_HIP_FORCE_DEV_KERNARG = "HIP_FORCE_DEV_KERNARG"
# the node's trusted comgr cache (quota/comgr_cache.py): code objects the HIP runtimes build at a
# process's first stream, compiled once by the DaemonSet's init container and mounted read-only
ENV_COMGR_CACHE = "AMD_COMGR_CACHE"
ENV_COMGR_CACHE_DIR = "AMD_COMGR_CACHE_DIR"
COMGR_CACHE_CONTAINER_DIR = "/run/gpushare/comgr-cache"
# the whole-pipeline cache in front of comgr (native/comgrcache), installed next to the shim
COMGR_ACTION_LIB_NAME = "libgpushare_comgrcache.so"
ENV_COMGR_ACTION_CACHE = "GPUSHARE_COMGR_ACTION_CACHE"
# container annotation (ContainerAllocateResponse.annotations): the host ledger directory key
# of this container, so the plugin can map an answer back to its ledger (quota/ledger.py)
CTR_ANNOTATION_LEDGER = "gpushare.amd.com/ledger"
ENV_GPU_UUID = "GPUSHARE_GPU_UUID"            # the physical GPU a container was given
ENV_ROCR_VISIBLE = "ROCR_VISIBLE_DEVICES"
# Compute isolation (--compute-isolation=cu, alloc/cuslots.py): queue CU masks read by ROCr / HIP.
ENV_HSA_CU_MASK = "HSA_CU_MASK"
ENV_ROC_CU_MASK = "ROC_GLOBAL_CU_MASK"
ENV_CU_SLOTS = "GPUSHARE_CU_SLOTS"              # the slot run, for the workload's information
POD_ANNOTATION_CU_SLOTS = "gpushare.amd.com/cu-slots"                  # written by the plugin
# label the MI355X extender sets with its annotations, before the bind: the node's plugin sees the
# pod coming (a label-selected watch) and prepares its Allocate answer ahead of the bind
POD_LABEL_NODE = "gpushare.amd.com/node"
POD_ANNOTATION_CU_SLOTS_REQUEST = "gpushare.amd.com/cu-slots-request"  # optional, set by the user
# Node annotation carrying the exported xGMI topology (JSON, see parallel/topology.py).
NODE_ANNOTATION_TOPOLOGY = "gpushare.amd.com/xgmi-topology"
NODE_ANNOTATION_HEALTH = "gpushare.amd.com/gpu-health"
# Node annotation carrying the unit of aliyun.com/gpu-mem on this node ("GiB" / "MiB"), so
# kubectl-inspect-gpushare labels it without guessing (the reference guesses, nodeinfo.go:228-244).
NODE_ANNOTATION_MEMORY_UNIT = "gpushare.amd.com/memory-unit"

# Environment used by the plugin itself (podmanager.go:33-58)
ENV_NODE_NAME = "NODE_NAME"
ENV_KUBECONFIG = "KUBECONFIG"

SA_TOKEN_FILE = "/var/run/secrets/kubernetes.io/serviceaccount/token"
SA_CA_FILE = "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt"


def plugin_socket(dir_: str | None = None) -> str:
    return os.path.join(dir_ or DEVICE_PLUGIN_PATH, PLUGIN_SOCKET_NAME)


def kubelet_socket(dir_: str | None = None) -> str:
    return os.path.join(dir_ or DEVICE_PLUGIN_PATH, KUBELET_SOCKET_NAME)

# Allocate reply trailing metadata: "<handler entry ns>,<handler exit ns>" (CLOCK_MONOTONIC)
HANDLER_STAMP_KEY = "gpushare-handler-ns"
