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
