"""Write-behind durability (round-1 review item 2): an Allocate answered before its
``ASSIGNED=true`` PATCH landed must survive an apiserver outage, a plugin kill and a restart.

Reference: ``allocate.go:132-152`` answers only after the PATCH landed; this build answers
first and journals the pending PATCH (``alloc/journal.py``).
"""
import json
import os
import time

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.alloc.journal import AllocJournal
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

from .test_allocate_engine import FakeClient, StaticSource, mkpod, req
from .test_units_and_model import gpu


def idx(adm, i=0):
    return int(dict(adm.responses[i].envs)[const.ENV_RESOURCE_INDEX])


def test_killed_plugin_lands_pending_patch_after_restart(tmp_path):
    """Apiserver drops the plugin's pod PATCHes; the plugin answers pod A (write-behind) and is
    SIGKILLed; a new plugin process starts while PATCHes still fail and admits an equal-size pod
    B: B gets its own GPU (A is never matched twice); when the apiserver recovers both pods end
    ASSIGNED=true."""
    journal = str(tmp_path / "alloc-journal.jsonl")
    with SimCluster([("n", "fake:2x4G")], plugin_mode="process",
                    extra_plugin_args=["--journal-path", journal]) as c:
        c.api.store.inject("assign_patch", 60)
        a, where_a, adm_a = c.run_pod(3, name="a")
        assert adm_a.error is None and idx(adm_a) == where_a[1]
        time.sleep(0.3)                     # the patcher is retrying against the outage
        assert O.annotations(c.client.get_pod("default", "a"))[const.ENV_ASSIGNED_FLAG] == "false"
        # the answer + pending patch record: in the journal, or (native server) in its fast file
        recs = [ln for f in (journal, journal + ".fast") if os.path.exists(f)
                for ln in open(f, errors="replace")]
        assert any('"op":"answer+patch"' in ln for ln in recs)
        # the kubelet has not reported A Running yet: A still looks like an assumed Pending pod
        c.client.patch_pod_status("default", "a", {"status": {"phase": "Pending"}})
        c.kill_plugin("n")
        c.restart_plugin("n")
        # the extender puts B (same size) on the other GPU (A's has 1 GiB left); the kubelet admits it
        b, where_b, adm_b = c.run_pod(3, name="b")
        assert where_b[1] != where_a[1]
        assert adm_b.error is None and idx(adm_b) == where_b[1]
        assert O.annotations(c.client.get_pod("default", "a"))[const.ENV_ASSIGNED_FLAG] == "false"
        assert c.api.store.requests["PATCH dropped"] >= 2
        c.api.store.inject("assign_patch", 0)
        for name in ("a", "b"):
            got = c.wait_assigned({"metadata": {"namespace": "default", "name": name}}, timeout=15)
            assert O.annotations(got)[const.ENV_ASSIGNED_FLAG] == "true", name
        # journal: every pending patch has its landing (written right after the PATCH returned:
        # the plugin process may still be at it when the annotation is already visible). Read
        # the files as they are: opening an AllocJournal would compact them under the plugin.
        def unlanded():                         # answers live in .fast, landings in the journal
            pend, landed = set(), set()
            for f in (journal, journal + ".fast"):
                if not os.path.exists(f):
                    continue
                for ln in open(f, "rb").read().split(b"\n"):
                    try:
                        e = json.loads(ln)
                    except ValueError:
                        continue
                    if e.get("op") in ("patch", "answer+patch"):
                        pend.add(e["uid"])
                    elif e.get("op") == "landed":
                        landed.add(e["uid"])
            return pend - landed

        t = time.monotonic() + 5
        while unlanded() and time.monotonic() < t:
            time.sleep(0.05)
        assert unlanded() == set()
    j = AllocJournal(journal)                   # the plugin is gone: the journal reader agrees
    assert j.unlanded() == []


def _model(n=2, gib=4):
    return DeviceModel([gpu(i, gib << 30) for i in range(n)], const.GIB)


def test_recovered_patch_skips_recreated_pod(tmp_path):
    """A journaled pending patch whose pod was deleted and re-created under the same name
    (new UID) is dropped, never applied to the new pod."""
    path = str(tmp_path / "j.jsonl")
    old = mkpod("web", 2, 0, 10, uid="uid-old")
    src = StaticSource([old])
    cl = FakeClient(src)
    cl.fail = RuntimeError("apiserver down")
    al = Allocator(_model(), src, cl, "node-a", AllocatorOptions(async_patch=True, journal_path=path))
    assert dict(al.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "0"
    al.close()                                   # "killed": the patch never landed
    new = mkpod("web", 2, 1, 20, uid="uid-new")
    src.pods[:] = [new]
    cl.fail = None
    cl.get_pod = lambda ns, name: next(p for p in src.pods if p["metadata"]["name"] == name)
    al2 = Allocator(_model(), src, cl, "node-a", AllocatorOptions(async_patch=True, journal_path=path))
    assert al2.flush_patches(5.0)
    assert not cl.patches                         # uid-old's patch never touched uid-new
    assert AllocJournal(path).unlanded() == []
    # the new pod is a normal candidate
    assert dict(al2.allocate(req(2)).container_responses[0].envs)[const.ENV_RESOURCE_INDEX] == "1"
    assert al2.flush_patches(5.0)
    assert [p[1] for p in cl.patches] == ["web"]
    al2.close()


def test_reconcile_repatches_answered_pod(tmp_path):
    """A pod this plugin answered that reads ASSIGNED=false (its patch was lost) is patched
    again by the reconcile pass; pods never answered are left alone."""
    path = str(tmp_path / "j.jsonl")
    a, other = mkpod("a", 2, 0, 10), mkpod("other", 2, 1, 20, phase="Running")
    src = StaticSource([a, other])
    cl = FakeClient(src)
    al = Allocator(_model(), src, cl, "node-a", AllocatorOptions(async_patch=True, journal_path=path,
                                                                   reconcile_s=3600))
    al.allocate(req(2))
    assert al.flush_patches(5.0)
    # an operator (or a stale writer) reverts the annotation
    for p in src.pods:
        if p["metadata"]["name"] == "a":
            p["metadata"]["annotations"][const.ENV_ASSIGNED_FLAG] = "false"
            p["status"]["phase"] = "Running"
    cl.get_pod = lambda ns, name: next(p for p in src.pods if p["metadata"]["name"] == name)
    assert al.reconcile() == 1
    assert al.flush_patches(5.0)
    assert [p[1] for p in cl.patches] == ["a", "a"]
    assert al.metrics.allocate_outcomes.value(outcome="patch_reconciled") == 1
    al.close()


def test_rebuild_keeps_inflight_claims(tmp_path):
    """A kubelet restart / SIGHUP rebuilds the plugin: the Allocator (claims, assigned pods,
    queued patches) is carried over, so a pod whose patch is still in flight is not matched
    again by the rebuilt plugin."""
    with SimCluster([("n", "fake:2x4G")]) as c:
        m = c.manager("n")
        c.api.store.inject("assign_patch", 60)
        _, where_a, adm_a = c.run_pod(3, name="a")
        c.client.patch_pod_status("default", "a", {"status": {"phase": "Pending"}})
        before = m.allocator
        c.nodes["n"].kubelet.registered.clear()      # wait for the *re*-registration below
        m.events.put(("signal", __import__("signal").SIGHUP))
        t = time.monotonic() + 10
        while m.restarts == 0 and time.monotonic() < t:
            time.sleep(0.01)
        assert c.nodes["n"].kubelet.registered.wait(10)
        assert m.allocator is before
        _, where_b, adm_b = c.run_pod(3, name="b")
        assert idx(adm_b) == where_b[1] != idx(adm_a)
        c.api.store.inject("assign_patch", 0)
        for name in ("a", "b"):
            got = c.wait_assigned({"metadata": {"namespace": "default", "name": name}}, timeout=10)
            assert O.annotations(got)[const.ENV_ASSIGNED_FLAG] == "true"


def test_mapped_journal_reload_and_compaction(tmp_path):
    """The journal is a MAP_SHARED file with a zero tail: records written by one instance are
    read back by the next (no close, as after a SIGKILL), and a full mapping compacts into a
    fresh file that keeps every live answer and unlanded patch."""
    from aliyun_gpushare_device_plugin_amd.alloc.journal import AllocJournal
    from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api

    path = str(tmp_path / "j.jsonl")
    j = AllocJournal(path, map_bytes=4096)
    resp = api.AllocateResponse()
    resp.container_responses.add(envs={"ALIYUN_COM_GPU_MEM_IDX": "1"})
    for i in range(40):                                   # ~4x the mapping: several compactions
        req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=[f"d{i}"])])
        j.record_pending(req, f"u{i}", resp, "default", f"p{i}", {"a": "b"})
        if i % 2:
            j.landed(f"u{i}")
    with open(path, "rb") as f:
        raw = f.read()
    assert raw.rstrip(b"\0").endswith(b"\n") and len(raw) >= 4096
    j2 = AllocJournal(path)                               # no close(): the writer was "killed"
    assert sorted(e["uid"] for e in j2.unlanded()) == sorted(f"u{i}" for i in range(0, 40, 2))
    assert all(j2.answered(f"u{i}") for i in range(40))
    req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=["d7"])])
    uid, got = j2.lookup(req)
    assert uid == "u7" and got().container_responses[0].envs["ALIYUN_COM_GPU_MEM_IDX"] == "1"


def test_prefault_survives_a_concurrent_compaction(tmp_path):
    """prefault (patcher thread) and a compaction (gRPC thread, journal full) used to
    race on the mapping: prefault raised ValueError('mmap closed') and killed the patcher."""
    import threading

    from aliyun_gpushare_device_plugin_amd.alloc.journal import AllocJournal
    from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api

    j = AllocJournal(str(tmp_path / "j.jsonl"), map_bytes=64 << 10)
    resp = api.AllocateResponse()
    resp.container_responses.add(envs={"K": "v" * 200})
    stop = threading.Event()
    errors = []

    def prefaulter():
        while not stop.is_set():
            try:
                j.prefault(ahead=64 << 10)
            except Exception as e:  # noqa: BLE001
                errors.append(e)
                return

    t = threading.Thread(target=prefaulter)
    t.start()
    try:
        for i in range(3000):             # ~1 KB records into a 64 KiB map: many compactions
            r = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=[f"d{i}"])])
            j.record(r, f"uid-{i % 50}", resp)
    finally:
        stop.set()
        t.join()
    assert errors == []
    j.close()


@pytest.mark.parametrize("seed,identity", [(s, False) for s in range(3, 7)] + [(1, True), (2, True)])
def test_chaos_churn_never_overcommits_and_every_patch_lands(tmp_path, seed, identity):
    """Randomised churn through the whole stack (extender, native server, engine, journal,
    placement truth) with faults mixed in: the plugin SIGKILLed and restarted, the apiserver
    dropping the plugin's PATCHes for a while; without admission identity equal-size pods also
    swap reservations and placement truth repairs them. Invariants: no GPU is ever given more than it
    has (by what the admitted containers were really answered), and once the faults stop every
    admitted pod ends ASSIGNED=true with nothing left unlanded in the journal."""
    import random

    rnd = random.Random(seed)
    journal = str(tmp_path / "j.jsonl")
    cap = 16
    with SimCluster([("n", "fake:2x16G")], plugin_mode="process", admission_identity=identity,
                    extra_plugin_args=["--journal-path", journal]) as c:
        c.extender.watch()
        live: dict = {}                                        # name -> (gpu answered, size)
        faults = {"kill": 0, "patch_outage": 0}
        for step in range(60):
            r = rnd.random()
            if step in (10, 35):
                r = 0.0                                        # at least two kills per run
            elif step in (5, 25):
                r = 0.1                                        # and two PATCH outages
            if r < 0.08:
                faults["kill"] += 1
                c.kill_plugin("n")
                c.restart_plugin("n")
            elif r < 0.16:
                faults["patch_outage"] += 1
                c.api.store.inject("assign_patch", rnd.uniform(0.2, 1.0))
            elif r < 0.40 and live:
                name = rnd.choice(sorted(live))
                c.delete_pod(c.client.get_pod("default", name))
                del live[name]
            else:
                size = rnd.choice([1, 2, 4, 8])
                pod, where, adm = c.run_pod(size)
                if where is None:
                    continue                                   # the extender found no room
                assert adm.error is None, adm.error
                g = int(adm.responses[0].envs[const.ENV_RESOURCE_INDEX])
                live[pod["metadata"]["name"]] = (g, size)
                used = {0: 0, 1: 0}
                for gg, s in live.values():
                    used[gg] += s
                assert max(used.values()) <= cap, (step, used)
        assert faults["kill"] >= 2 and faults["patch_outage"] >= 2 and len(live) >= 1
        c.api.store.inject("assign_patch", 0)
        for name in live:
            got = c.wait_assigned({"metadata": {"namespace": "default", "name": name}}, timeout=20)
            assert O.annotations(got)[const.ENV_ASSIGNED_FLAG] == "true", name
