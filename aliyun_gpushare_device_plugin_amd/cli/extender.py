"""``gpushare-scheduler-extender`` — an MI355X-aware scheduler extender for ``aliyun.com/gpu-mem``.

The reference plugin relies on the external Go ``gpushare-scheduler-extender`` (linked from
its ``README.md:14``) for the bin-packing decision; it writes the ``ALIYUN_COM_GPU_MEM_*``
annotations the plugin consumes. This is a drop-in for it with the same wire
behaviour (kube-scheduler extender ``filter`` / ``bind`` verbs, best-fit per GPU by HBM,
the same annotations) plus what MI355X needs:

* TP groups (pods labelled ``gpushare.amd.com/tp-group`` / ``tp-size``) get GPUs that are
  pairwise one-hop xGMI per the topology the plugin exports, reserved for the whole group when
  its first member binds (``extender/core.py`` ``bind_member``);
* unhealthy GPUs (the plugin's health annotation) are never chosen;
* placement follows the plugin's placement-truth rewrites (pod informer, ``update``);
* ``--leader-elect``: several replicas, one serving at a time (a Lease, ``extender/leader.py``);
  the others keep a warm ledger and take over when the leader stops renewing.

Configure kube-scheduler with ``deploy/scheduler-extender.yaml`` (KubeSchedulerConfiguration
``extenders`` entry: urlPrefix ``http://<svc>:39999/gpushare-scheduler``, ``filterVerb: filter``,
``bindVerb: bind``, ``managedResources: aliyun.com/gpu-mem``).
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading

from ..cluster.client import build_client
from ..extender import Extender, LeaderElector, serve_http
from ..utils import log


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="gpushare-scheduler-extender", description=__doc__.splitlines()[0])
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=39999)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--apiserver", default=None, help="apiserver URL (default: kubeconfig / in-cluster)")
    p.add_argument("--policy", default="binpack", choices=("binpack", "spread"))
    p.add_argument("--resync", type=float, default=30.0, help="seconds between full node/pod re-syncs")
    p.add_argument("--group-ttl", type=float, default=300.0,
                   help="seconds a TP group's reserved GPUs wait for its remaining members")
    p.add_argument("--leader-elect", action="store_true",
                   help="run as one of several replicas: only the Lease holder answers filter/bind")
    p.add_argument("--leader-elect-namespace", default="kube-system")
    p.add_argument("--leader-elect-name", default="gpushare-scheduler-extender")
    p.add_argument("--leader-elect-identity", default=None, help="default: $POD_NAME or the hostname, plus a random suffix")
    p.add_argument("--leader-elect-lease-duration", type=float, default=15.0)
    p.add_argument("--leader-elect-renew-deadline", type=float, default=10.0)
    p.add_argument("--leader-elect-retry-period", type=float, default=2.0)
    p.add_argument("-v", "--v", type=int, default=0)
    return p


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    log.setup(verbosity=a.v, buffered=True)
    client = build_client(a.kubeconfig, a.apiserver)
    ext = Extender(client, a.policy, a.group_ttl)
    ext.sync()
    ext.watch()
    if a.leader_elect:
        import os
        import socket
        import uuid

        ident = a.leader_elect_identity or f"{os.environ.get('POD_NAME') or socket.gethostname()}_{uuid.uuid4().hex[:8]}"
        # a new leader counts every bind the previous one made before it answers (sync)
        ext.elector = LeaderElector(client, a.leader_elect_namespace, a.leader_elect_name, ident,
                                    a.leader_elect_lease_duration, a.leader_elect_renew_deadline,
                                    a.leader_elect_retry_period, on_start=ext.sync).start()
    srv = serve_http(ext, a.host, a.port)
    log.info("gpushare scheduler extender on %s:%d (%d shared-GPU nodes)", a.host, srv.server_address[1],
             len(ext.nodes))
    print(f"listening {srv.server_address[1]}", flush=True)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    while not stop.wait(a.resync):
        try:
            ext.sync()
        except Exception as e:  # noqa: BLE001 - keep serving on the last good view
            log.warning("resync failed: %s", e)
    if ext.elector is not None:
        ext.elector.stop(release=True)
    ext.stop_watch()
    srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
