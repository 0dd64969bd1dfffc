"""The per-node HBM broker launcher (``cli/hbmbroker.py``) on CPU, with a stand-in broker binary:
one broker per GPU of the node, found by PCI address, and a broker that dies is started again."""
from __future__ import annotations

import json
import os
import stat
import sys
import time

from aliyun_gpushare_device_plugin_amd.cli import hbmbroker as cli
from aliyun_gpushare_device_plugin_amd.device.smi import SMI

STANDIN = """#!{py}
import json, sys, time
a = sys.argv[1:]
sock = a[a.index("--socket") + 1]
bdf = a[a.index("--pci-bus-id") + 1]
open(sock + ".args", "a").write(json.dumps(a) + "\\n")
print(json.dumps({{"ready": True, "socket": sock, "granules": 4, "granule_bytes": 1 << 30}}), flush=True)
time.sleep(600)
"""


def test_launcher_runs_one_broker_per_gpu_and_restarts_a_dead_one(tmp_path, monkeypatch):
    exe = tmp_path / "standin-broker"
    exe.write_text(STANDIN.format(py=sys.executable))
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("GPUSHARE_HBM_BROKER_EXE", str(exe))
    d = tmp_path / "hbm"
    d.mkdir()
    with SMI("fake:2x64G") as s:
        gpus = [s.device(i) for i in range(s.count())]
    brokers = {g.index: cli.HBMBroker.for_gpu(str(d), g.index, pci_bus_id=g.bdf) for g in gpus}
    sup = cli.Supervisor(brokers, backoff_s=0.1)
    try:
        sup.start()
        for g in gpus:
            args = json.loads((d / f"gpu{g.index}" / f"hbm{g.index}.sock.args").read_text().splitlines()[0])
            assert args[args.index("--pci-bus-id") + 1] == g.bdf        # by PCI address, not HIP order
            # the pod socket in the GPU's own directory, the admin socket apart (never mounted)
            assert args[args.index("--socket") + 1] == str(d / f"gpu{g.index}" / f"hbm{g.index}.sock")
            assert args[args.index("--admin-socket") + 1] == str(d / "admin" / f"hbm{g.index}.sock")
        assert oct(os.stat(d / "admin").st_mode & 0o777) == "0o700"
        brokers[1].proc.kill()
        brokers[1].proc.wait()
        sup.watch_once()
        assert sup.restarts == {0: 0, 1: 1}
        assert brokers[1].proc.poll() is None
        assert len((d / "gpu1" / "hbm1.sock.args").read_text().splitlines()) == 2
    finally:
        sup.stop()
    assert all(b.proc is None for b in brokers.values())
