"""Round-3 review item 4: HBM shares hold for a tenant that drops the quota shim, by default.

With no dmem cgroup controller (the MI355X test boxes' kernel, ``profiles/r3/dmem_probe.txt``)
the default ``--quota-enforcement=auto`` runs the watchdog in kill mode — but only with the
kubelet pod-resources API (placement truth): without it a swapped admission leaves annotations
crossed, so kill is downgraded to report and ``/readyz`` says the shares are not enforced.
Reference: ``allocate.go:125-127`` (isolation is on unless the node label disables it)."""
import os

from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

NATIVE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aliyun_gpushare_device_plugin_amd",
                      "_native")


def _mode(mgr):
    return {m: mgr.metrics.enforcement_mode.value(mode=m) for m in ("dmem", "kill", "report", "off")}


def test_auto_enforces_by_kill_with_placement_truth():
    with SimCluster([("n", "fake:2x8G")], shim_host_dir=NATIVE) as c:
        mgr = c.manager("n")
        assert mgr.cfg.quota_enforcement == "auto"
        assert mgr.enforcement == "kill" and mgr.watchdog is not None and mgr.watchdog.mode == "kill"
        assert _mode(mgr) == {"dmem": 0, "kill": 1, "report": 0, "off": 0}
        assert mgr.readiness() == (True, "ok")
        # the watchdog reads the allocator's view and in-flight state
        assert mgr.watchdog.settled.__self__ is mgr.allocator


def test_no_pod_resources_downgrades_kill_and_reports_not_ready():
    with SimCluster([("n", "fake:2x8G")], shim_host_dir=NATIVE, placement_truth=False) as c:
        mgr = c.manager("n")
        assert mgr.enforcement == "report" and mgr.watchdog.mode == "report"
        assert _mode(mgr)["report"] == 1 and _mode(mgr)["kill"] == 0
        ok, why = mgr.readiness()
        assert not ok and "not enforced" in why


def test_explicit_kill_without_pod_resources_is_refused():
    with SimCluster([("n", "fake:1x8G")], shim_host_dir=NATIVE, placement_truth=False) as c:
        mgr = c.manager("n")
        mgr.cfg.quota_enforcement = "kill"
        assert mgr._enforcement() == "report" and mgr.enforcement == "report"


def test_kernel_dmem_limits_take_precedence():
    class Dmem:
        def available(self):
            return True

    with SimCluster([("n", "fake:1x8G")], shim_host_dir=NATIVE) as c:
        mgr = c.manager("n")
        mgr.dmem = Dmem()
        assert mgr._enforcement() == "report"         # the watchdog only reports: the kernel limits
        assert mgr.enforcement == "dmem" and _mode(mgr)["dmem"] == 1 and mgr.readiness()[0]


def test_settled_tracks_answers_and_placement_passes():
    """A pod is "settled" for the watchdog only after a placement pass has seen the latest
    answer and its ASSIGNED patch landed."""
    with SimCluster([("n", "fake:2x8G")]) as c:
        mgr = c.manager("n")
        al = mgr.allocator
        pod, where, adm = c.run_pod(4)
        uid = pod["metadata"]["uid"]
        assert al.flush_patches(5.0)
        al._drain_post()
        if al._placed_at >= al._last_grant:          # a periodic pass may already have run
            al._placed_at = 0.0
        assert not al.settled(uid)
        al.reconcile_placement()
        assert al.settled(uid)
        al.podres, podres = None, al.podres
        try:
            assert not al.settled(uid)                # no placement truth: never settled
        finally:
            al.podres = podres
