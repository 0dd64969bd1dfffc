"""``gpushare-hbm-brokers`` — run and supervise one HBM broker per GPU of the node.

Each broker (``native/hbmbroker``, ``gpushare-hbm-broker``) holds its GPU's shareable HBM as VMM
granules and lends each pod its own, zeroed between pods (``docs/HBM_TURNOVER.md``). The device
plugin, started with ``--hbm-broker-dir`` on the same directory, grants every shared container its
granules. GPU ``i`` of the plugin (its SMI order) gets the pod socket ``<dir>/gpu<i>/hbm<i>.sock``
and the admin socket ``<dir>/admin/hbm<i>.sock`` (``quota/hbmbroker.py`` has the layout), and
the broker finds its HIP device by that GPU's PCI address, because HIP and SMI orders are not
promised to agree.

Sizing: each broker is sized for its GPU less ``--reserve-gib``. With ``--start-empty`` (the
DaemonSet) it holds nothing until the plugin's granter sizes it: the whole size, or nothing on a
``cgpu.disable.isolation=true`` node (``SIZE``), so such a node's GPUs stay the driver's. Free
granules go back to the driver when it runs short (``--low-water-gib``).

A broker that exits is started again after ``--restart-backoff`` seconds, with a new boot id: the
plugin sees it on its next poll and grants the new instance every live pod's token again, so a
container that restarts afterwards gets its granules. Pods that held granules of the dead broker
keep what they mapped until they exit (docs/HBM_TURNOVER.md, exporter death). A pod whose first
allocation comes while its broker is down waits for it (the shim retries the socket), within
``GPUSHARE_HBM_WAIT_S``.

No counterpart in the reference (``pkg/gpu/nvidia/allocate.go:114-127`` leaves isolation and
memory to cGPU).
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import threading
import time

from ..device.smi import SMI
from ..quota.hbmbroker import HBMBroker
from ..utils import log


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="gpushare-hbm-brokers", description=__doc__.splitlines()[0])
    p.add_argument("--dir", default="/var/run/gpushare/hbm", help="socket directory (the plugin's --hbm-broker-dir)")
    p.add_argument("--smi-backend", default="auto")
    p.add_argument("--gpu-indices", default="", help="comma-separated plugin GPU indices (default: all)")
    p.add_argument("--reserve-gib", type=float, default=12.0,
                   help="HBM each broker leaves to the driver (the pods' runtimes allocate some themselves)")
    p.add_argument("--granule-mib", type=int, default=1024)
    p.add_argument("--wait-s", type=float, default=30.0, help="how long a pod's TAKE waits for its granules")
    p.add_argument("--ungranted-wait-s", type=float, default=10.0,
                   help="how long a TAKE whose grant has not arrived waits (the plugin re-grants within a poll)")
    p.add_argument("--release-policy", default="auto", choices=("auto", "refs", "exit"),
                   help="when a released granule may be lent again (hbmbroker.cpp): refs = no dma-buf reference "
                        "left outside the broker, exit = the holder's process is gone; auto = refs where the "
                        "kernel counts them")
    p.add_argument("--scrub-chunk", type=int, default=8,
                   help="granules zeroed per scrub event: a released pod's granules are lent again chunk by chunk")
    p.add_argument("--scrub-kernel", default="",
                   help="the broker's scrub code object (default: gpushare-hbm-scrub.co next to the broker); "
                        "without it the broker zeroes with hipMemsetAsync")
    p.add_argument("--restart-backoff", type=float, default=2.0)
    p.add_argument("--start-empty", action="store_true",
                   help="brokers hold nothing until the plugin sizes them (SIZE): on a cgpu.disable.isolation node "
                        "they never take the GPU's HBM from the driver")
    p.add_argument("--low-water-gib", type=float, default=-1.0,
                   help="free granules go back to the driver when it has less than this free (default: half the "
                        "reserve); the brokers grow again once it has more than the reserve")
    return p


class Supervisor:
    def __init__(self, brokers: dict[int, HBMBroker], backoff_s: float = 2.0):
        self.brokers, self.backoff_s = brokers, backoff_s
        self.restarts = {i: 0 for i in brokers}
        self._stop = threading.Event()

    def start(self) -> None:
        for i, b in self.brokers.items():
            info = b.start()
            log.info("hbm broker of GPU %d: %s granules of %s bytes at %s", i, info.get("granules"),
                     info.get("granule_bytes"), b.socket_path)

    def watch_once(self) -> None:
        for i, b in self.brokers.items():
            p = b.proc
            if p is not None and p.poll() is None:
                continue
            rc = p.returncode if p is not None else None
            log.warning("hbm broker of GPU %d exited (%s); starting it again", i, rc)
            self.restarts[i] += 1
            b.proc = None
            try:
                b.start()
            except Exception as e:  # noqa: BLE001 - retried on the next pass
                log.warning("hbm broker of GPU %d did not start: %s", i, e)

    def run(self) -> None:
        while not self._stop.wait(self.backoff_s):
            self.watch_once()

    def stop(self) -> None:
        self._stop.set()
        for b in self.brokers.values():
            b.stop()


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    log.setup(buffered=True)
    os.makedirs(a.dir, exist_ok=True)
    os.chmod(a.dir, 0o755)
    want = {int(x) for x in a.gpu_indices.split(",") if x.strip()}
    with SMI(a.smi_backend) as s:
        gpus = [s.device(i) for i in range(s.count())]
    extra = ["--ungranted-wait-s", str(a.ungranted_wait_s), "--release-policy", a.release_policy,
             "--scrub-chunk", str(a.scrub_chunk)]
    if a.start_empty:
        extra.append("--start-empty")
    if a.low_water_gib >= 0:
        extra += ["--low-water-gib", str(a.low_water_gib)]
    if a.scrub_kernel:
        extra += ["--scrub-kernel", a.scrub_kernel]
    brokers = {g.index: HBMBroker.for_gpu(a.dir, g.index, pci_bus_id=g.bdf, reserve_gib=a.reserve_gib,
                                          granule_mib=a.granule_mib, wait_s=a.wait_s, extra_args=extra)
               for g in gpus if not want or g.index in want}
    if not brokers:
        log.error("no GPU to run an HBM broker for")
        return 1
    sup = Supervisor(brokers, a.restart_backoff)
    signal.signal(signal.SIGTERM, lambda *_: sup._stop.set())
    signal.signal(signal.SIGINT, lambda *_: sup._stop.set())
    try:
        sup.start()
        sup.run()
    finally:
        sup.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
