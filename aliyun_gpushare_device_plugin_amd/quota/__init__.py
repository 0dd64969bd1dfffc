"""Per-container HBM quota enforcement: configuration of the HIP intercept shim.

The reference delegates isolation to Alibaba's external cGPU module, driven purely by the
``ALIYUN_COM_GPU_MEM_*`` env contract and switched off by ``CGPU_DISABLE``
(``allocate.go:114-129``). On MI355X the plugin ships its own enforcement: the C++ LD_PRELOAD
shim ``libgpushare_hipquota.so`` (native/hipshim/hipquota.cpp) reads the same env vars and
caps every HIP allocation path at ``CONTAINER / DEV × real HBM bytes``. This module builds
the Allocate-response pieces that inject it (a read-only mount + ``LD_PRELOAD``) and the
environment for running a workload under it locally.
"""
from __future__ import annotations

import dataclasses
import os

from .. import const
from ..utils.native import lib_path

GRANULE_BYTES = 2 << 20  # hipMalloc rounds every allocation to 2 MiB on MI355X (measured)


@dataclasses.dataclass
class ShimConfig:
    host_dir: str                      # directory on the node holding libgpushare_hipquota.so
    container_dir: str = const.SHIM_CONTAINER_DIR
    enabled: bool = True

    @property
    def container_lib(self) -> str:
        return os.path.join(self.container_dir, const.SHIM_LIB_NAME)

    @classmethod
    def in_tree(cls) -> "ShimConfig":
        return cls(host_dir=os.path.dirname(lib_path("hipshim")))


def ledger_name(pod_uid: str, container_slot: int) -> str:
    """POSIX shm name shared by all processes of one container (quota is per container)."""
    safe = "".join(filter(str.isalnum, pod_uid))[:40] or "anon"
    return f"/gpushare-{safe}-{container_slot}"


def shim_env(container_units: int, dev_units: int, ledger: str, lib: str | None = None,
             quota_bytes: int | None = None, log_level: int | None = None) -> dict[str, str]:
    """Environment to run one process under the quota shim (used by tests and demos)."""
    env = {
        const.ENV_RESOURCE_BY_CONTAINER: str(container_units),
        const.ENV_RESOURCE_BY_DEV: str(dev_units),
        const.ENV_SHIM_LEDGER: ledger,
        const.ENV_LD_PRELOAD: lib or lib_path("hipshim"),
    }
    if quota_bytes is not None:
        env[const.ENV_SHIM_QUOTA_BYTES] = str(int(quota_bytes))
    if log_level is not None:
        env[const.ENV_SHIM_LOG] = str(log_level)
    return env
