"""Scheduler-extender HA (``extender/leader.py``, ``--leader-elect``): a Lease elects one serving
replica; followers answer 503 and stay unready; a crashed leader is replaced once its lease
expires, a released one at once; a leader cut off from the apiserver steps down before anyone
else may take over; the new leader re-syncs its ledger first, so no HBM is handed out twice."""
import json
import time
import urllib.error
import urllib.request

import pytest

from aliyun_gpushare_device_plugin_amd.cluster.client import APIClient, KubeConfig
from aliyun_gpushare_device_plugin_amd.extender import Extender, LeaderElector, serve_http
from aliyun_gpushare_device_plugin_amd.sim.apiserver import FakeAPIServer
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

FAST = dict(lease_s=1.0, renew_s=0.6, retry_s=0.1)


def _elector(url, ident, **kw):
    return LeaderElector(APIClient(KubeConfig(url)), "kube-system", "gpushare-scheduler-extender", ident,
                         **dict(FAST, **kw))


def _until(cond, timeout=5.0):
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if cond():
            return True
        time.sleep(0.02)
    return cond()


def _lease(api):
    return api.store.leases[("kube-system", "gpushare-scheduler-extender")]


def test_exactly_one_leader_and_failover_after_a_crash():
    with FakeAPIServer() as api:
        a, b = _elector(api.url, "a").start(), _elector(api.url, "b").start()
        try:
            assert _until(lambda: a.is_leader() or b.is_leader())
            for _ in range(20):                               # never two at once
                assert not (a.is_leader() and b.is_leader())
                time.sleep(0.05)
            lead, other = (a, b) if a.is_leader() else (b, a)
            assert _lease(api)["spec"]["holderIdentity"] == lead.identity
            t0 = time.monotonic()
            lead.stop(release=False)                          # crash: no release
            assert _until(other.is_leader, 5.0)
            waited = time.monotonic() - t0
            assert waited >= 0.9 * FAST["lease_s"]            # not before the lease ran out
            spec = _lease(api)["spec"]
            assert spec["holderIdentity"] == other.identity and spec["leaseTransitions"] >= 1
        finally:
            a.stop()
            b.stop()


def test_a_released_lease_is_taken_at_once():
    with FakeAPIServer() as api:
        a = _elector(api.url, "a", lease_s=5.0, renew_s=3.0)
        a.step()
        assert a.is_leader()
        b = _elector(api.url, "b", lease_s=5.0, renew_s=3.0)
        b.step()
        assert not b.is_leader()
        a.stop(release=True)
        b.step()
        assert b.is_leader() and _lease(api)["spec"]["holderIdentity"] == "b"


def test_a_leader_cut_off_from_the_apiserver_steps_down_first():
    stopped = []
    with FakeAPIServer() as api:
        a = _elector(api.url, "a", on_stop=lambda: stopped.append(time.monotonic()))
        b = _elector(api.url, "b")
        a.step()
        assert a.is_leader()
        api.store.inject("lease", 2.0)                        # a cannot renew, b cannot read
        t0 = time.monotonic()
        while time.monotonic() - t0 < 1.2:
            a.step()
            b.step()
            time.sleep(0.05)
        assert stopped and stopped[0] - t0 < FAST["lease_s"]  # a stepped down within its renew deadline
        assert not a.is_leader() and not b.is_leader()
        api.store.inject("lease", 0)
        assert _until(lambda: (a.step(), b.step(), a.is_leader() or b.is_leader())[-1])


def test_clock_skew_cannot_hand_over_a_live_lease():
    """The holder's renewTime is never compared with local time: a follower whose clock runs far
    ahead still waits a full lease duration without seeing the record change."""
    with FakeAPIServer() as api:
        a = _elector(api.url, "a", lease_s=5.0, renew_s=3.0)
        a.step()
        skew = [10_000.0]
        b = _elector(api.url, "b", lease_s=5.0, renew_s=3.0, clock=lambda: time.monotonic() + skew[0])
        for _ in range(5):
            a.step()
            b.step()
            assert a.is_leader() and not b.is_leader()


def test_only_the_leader_serves_and_a_new_leader_resyncs_before_it_binds():
    """Two extender replicas behind HTTP. The follower answers 503 (readyz and filter). A binds a
    pod through HTTP, then crashes; B (whose ledger has not seen that bind — no pod watch here)
    re-syncs when it takes over, so it does not put a second full-GPU pod on the same GPU."""
    with SimCluster([("n", "fake:1x8G")]) as c:
        exts, srvs = [], []
        for ident in ("a", "b"):
            e = Extender(APIClient(KubeConfig(c.api_url)))
            e.sync()
            e.elector = _elector(c.api_url, ident, on_start=e.sync)
            exts.append(e)
            srvs.append(serve_http(e))
        ea, eb = exts
        ea.elector.step()
        eb.elector.step()
        assert ea.serving() and not eb.serving()

        def get(srv, path):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{srv.server_address[1]}{path}", timeout=5) as r:
                    return r.status
            except urllib.error.HTTPError as e:
                return e.code

        def post(srv, path, body):
            req = urllib.request.Request(f"http://127.0.0.1:{srv.server_address[1]}{path}",
                                         data=json.dumps(body).encode(), method="POST")
            try:
                with urllib.request.urlopen(req, timeout=5) as r:
                    return r.status, json.loads(r.read())
            except urllib.error.HTTPError as e:
                return e.code, json.loads(e.read())

        try:
            assert get(srvs[0], "/readyz") == 200 and get(srvs[1], "/readyz") == 503
            assert get(srvs[1], "/healthz") == 200
            p1 = c.create_pod(8, name="p1")
            args = {"Pod": p1, "NodeNames": ["n"]}
            assert post(srvs[1], "/gpushare-scheduler/filter", args)[0] == 503
            code, res = post(srvs[0], "/gpushare-scheduler/filter", args)
            assert code == 200 and res["NodeNames"] == ["n"]
            code, res = post(srvs[0], "/gpushare-scheduler/bind",
                             {"PodName": "p1", "PodNamespace": "default", "Node": "n"})
            assert code == 200 and res["Error"] == ""
            assert eb.usage()["n"]["used"] == [0]             # B has not seen the bind
            ea.elector.stop(release=False)                    # A crashes
            assert _until(lambda: (eb.elector.step(), eb.serving())[-1], 5.0)
            assert eb.usage()["n"]["used"] == [8]             # re-synced before serving
            assert get(srvs[1], "/readyz") == 200
            p2 = c.create_pod(8, name="p2")
            code, res = post(srvs[1], "/gpushare-scheduler/filter", {"Pod": p2, "NodeNames": ["n"]})
            assert code == 200 and res["NodeNames"] == []     # the GPU is full: no double booking
        finally:
            for s in srvs:
                s.shutdown()
            eb.elector.stop()


def test_cli_flags_and_manifest():
    from aliyun_gpushare_device_plugin_amd.cli.extender import build_parser

    a = build_parser().parse_args(["--leader-elect", "--leader-elect-lease-duration", "20"])
    assert a.leader_elect and a.leader_elect_lease_duration == 20.0
    import os

    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = list(yaml.safe_load_all(open(os.path.join(root, "deploy", "scheduler-extender.yaml"))))
    dep = next(d for d in docs if d and d.get("kind") == "Deployment")
    ctr = dep["spec"]["template"]["spec"]["containers"][0]
    assert dep["spec"]["replicas"] >= 2 and "--leader-elect" in ctr["command"]
    assert ctr["readinessProbe"]["httpGet"]["path"] == "/readyz"
    role = next(d for d in docs if d and d.get("kind") == "ClusterRole")
    assert any("leases" in r["resources"] and {"get", "create", "update"} <= set(r["verbs"]) for r in role["rules"])


def test_bad_timings_are_refused():
    with pytest.raises(ValueError):
        LeaderElector(None, "ns", "n", "x", lease_s=5, renew_s=6, retry_s=1)


def test_a_slow_renewal_does_not_extend_the_leaders_term():
    """the leader's renewal counts from when it started, not when its PUT returned;
    a follower dates its observation from when its GET returned."""
    clock = [100.0]

    class SlowClient:
        def __init__(self, inner, delay):
            self.inner, self.delay = inner, delay
            self.timeouts = []

        def request(self, method, path, body=None, timeout=None):
            self.timeouts.append(timeout)
            r = self.inner.request(method, path, body=body)
            clock[0] += self.delay                    # the request took this long
            return r

    api = FakeAPIServer()
    api.start()
    try:
        from aliyun_gpushare_device_plugin_amd.cluster.client import APIClient, KubeConfig
        from aliyun_gpushare_device_plugin_amd.extender.leader import LeaderElector

        slow = SlowClient(APIClient(KubeConfig(api.url)), delay=4.0)
        le = LeaderElector(slow, "kube-system", "x", "a", lease_s=15.0, renew_s=10.0, retry_s=2.0, clock=lambda: clock[0])
        t0 = clock[0]
        le.step()                                      # POST (create) took 4 s
        assert le._leader and le._last_renew == t0
        assert all(t == 4.0 for t in slow.timeouts)    # (renew 10 - retry 2) / 2
        t1 = clock[0]
        le.step()                                      # GET + PUT: 8 s, started at t1
        assert le._last_renew == t1 and clock[0] - le._last_renew == 8.0
        f = LeaderElector(SlowClient(APIClient(KubeConfig(api.url)), delay=3.0), "kube-system", "x", "b",
                          lease_s=15.0, renew_s=10.0, retry_s=2.0, clock=lambda: clock[0])
        before = clock[0]
        assert f.try_acquire_or_renew() is False
        assert f._observed_at == before + 3.0          # when the GET returned
    finally:
        api.stop()
