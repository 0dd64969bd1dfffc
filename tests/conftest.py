"""Shared pytest configuration.

Markers:
  gpu  — needs a real MI355X (runs via `pytest -m gpu` on the GPU box); everything else must
         pass on a CPU-only host.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires a real MI355X GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native_gpuinfo():
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built
    return ensure_built("gpuinfo")


@pytest.fixture(scope="session")
def native_shim():
    from aliyun_gpushare_device_plugin_amd.utils.native import ensure_built
    return ensure_built("hipshim")


@pytest.fixture(autouse=True)
def _quiet_logs():
    import logging
    from aliyun_gpushare_device_plugin_amd.utils import log
    log.logger.setLevel(logging.WARNING)
    yield


@pytest.fixture(scope="session")
def stub_runtime(tmp_path_factory):
    """A directory with the stub HIP runtime (tests/native/fake_hip.c, soname libamdhip64.so.7),
    the shim test driver linked against it, and the HBM broker linked against it: everything a
    CPU rehearsal of the broker path runs (the real quota shim is preloaded on top)."""
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    d = tmp_path_factory.mktemp("stubrt")
    lib = d / "libamdhip64.so.7"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-Wl,-soname,libamdhip64.so.7", "-o", str(lib),
                    os.path.join(here, "native", "fake_hip.c")], check=True)
    subprocess.run(["gcc", "-O1", "-pthread", "-o", str(d / "shim_driver"), os.path.join(here, "native", "shim_driver.c"),
                    str(lib), f"-Wl,-rpath,{d}", "-ldl"], check=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o",
                    str(d / "gpushare-hbm-broker"), os.path.join(ROOT, "native", "hbmbroker", "hbmbroker.cpp"), str(lib),
                    f"-Wl,-rpath,{d}"], check=True)
    return str(d)
