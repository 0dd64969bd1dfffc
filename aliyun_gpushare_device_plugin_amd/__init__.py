"""MI355X-native GPU-sharing Kubernetes device plugin (aliyun.com/gpu-mem compatible).

Layer map (re-designed for MI355X):
  L0 device/smi.py       -> native/gpuinfo (C++: librocm_smi64 + amdgpu/KFD sysfs)
  L1 device/model.py     physical GPU -> fake memory-unit devices
  L2 cluster/            apiserver client, node status, pod watch cache, kubelet client
  L3 plugin/server.py    kubelet v1beta1 DevicePlugin gRPC server; alloc/ Allocate engine
  L4 plugin/manager.py   lifecycle (inotify, signals, restart), device/health.py
  L5 cli/main.py         flags / entry point
  L6 cli/inspect.py      kubectl-inspect-gpushare; cli/podgetter.py
  quota/ + native/hipshim  per-container HBM quota (LD_PRELOAD HIP interposer)
  ops/ + models/           HIP/CDNA4 kernels and the PyTorch-ROCm demo workloads
  parallel/                xGMI topology export, TP-group placement, RCCL demo
  sim/                     fake apiserver / kubelet / extender for CPU-only end-to-end runs
"""
__version__ = "0.1.0"
