"""Allocate fast path (prepared answers) — same decisions as the full match, less work.

The engine keeps every candidate pod's single-container answer serialized ahead of time;
when the watch cache has not changed since, Allocate only picks the first eligible candidate
of the request's size, appends its journal record to the mapped file and returns the bytes.
"""
import time

import pytest

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc.journal import AllocJournal
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster


SERVERS = ["python", "native"]    # grpcio + the engine's fast path; libgpushare_dpserver's table


def _settle(al, timeout=5.0, quiet=0.1):
    """Wait until the prepared answers match the pod cache (the engine's own table, or the one
    published to the native server) and the cache has not changed for ``quiet`` seconds (the fake
    kubelet's own status updates of a just-bound pod come in after the bind)."""
    t = time.monotonic() + timeout
    since, seen = time.monotonic(), None
    while time.monotonic() < t:
        v = al.pods.pending_version
        if v != seen:
            since, seen = time.monotonic(), v
        if al.native is not None:
            current = al._published == (v, al._gen)
        else:
            f = al._fast
            current = f is not None and f.version == v and f.gen == al._gen
        if current and time.monotonic() - since >= quiet:
            return True
        time.sleep(0.005)
    return False


def _fast_count(al):
    return al.metrics.allocate_latency.count(phase="native" if al.native is not None else "fast")


def _envs(r):
    e = dict(r.envs)
    e.pop(const.ENV_SHIM_LEDGER, None)
    return e


@pytest.mark.parametrize("server", SERVERS)
def test_fast_path_answers_like_the_full_path(tmp_path, server):
    with SimCluster([("n", "fake:2x16G")], shim_host_dir=str(tmp_path), grpc_server=server) as c:
        al = c.manager("n").allocator
        pods = [c.create_pod(s, name=f"p{i}") for i, s in enumerate((4, 8))]
        places = [c.schedule(p) for p in pods]
        assert _settle(al)
        adm = c.admit(pods[0])
        assert adm.error is None
        assert _fast_count(al) == 1
        env = _envs(adm.responses[0])
        assert env[const.ENV_RESOURCE_INDEX] == str(places[0][1])
        assert env[const.ENV_RESOURCE_BY_CONTAINER] == env[const.ENV_RESOURCE_BY_POD] == "4"
        assert {d.container_path for d in adm.responses[0].devices} >= {"/dev/kfd"}
        got = c.wait_assigned(pods[0])
        assert O.annotations(got)[const.ENV_ASSIGNED_FLAG] == "true"
        # the same pod answered by the full path (fast path off) carries the same envs
        al.opts.fast_path = False
        al._fast = None
        time.sleep(1.2)                        # the prepare loop publishes an empty native table
        adm2 = c.admit(pods[1])
        assert _fast_count(al) == 1
        assert _envs(adm2.responses[0])[const.ENV_RESOURCE_INDEX] == str(places[1][1])
        assert set(_envs(adm2.responses[0])) == set(env)


@pytest.mark.parametrize("server", SERVERS)
def test_fast_path_defers_to_identity_on_ambiguity(server):
    """Two pending pods of the same size: the fast path steps aside and admission identity
    (pod-resources) gives the kubelet's pod its own reservation."""
    with SimCluster([("n", "fake:2x8G")], grpc_server=server) as c:
        al = c.manager("n").allocator
        a, b = c.create_pod(8, name="a"), c.create_pod(8, name="b")
        assert c.schedule(a)[1] == 0 and c.schedule(b)[1] == 1
        assert _settle(al)
        adm = c.admit(b)
        assert int(adm.responses[0].envs[const.ENV_RESOURCE_INDEX]) == 1
        assert _fast_count(al) == 0
        assert al.metrics.allocate_outcomes.value(outcome="identified") == 1
        c.wait_assigned(b)                     # b's ASSIGNED patch has landed in the pod cache
        assert _settle(al)
        adm = c.admit(a)                       # now unambiguous: fast
        assert int(adm.responses[0].envs[const.ENV_RESOURCE_INDEX]) == 0
        assert _fast_count(al) == 1


def test_fast_records_survive_a_crash(tmp_path):
    """A fast-path record (answer + pending patch, request as wire bytes) is recovered by the
    next plugin instance: the patch is re-queued and a retried Allocate replays the answer."""
    path = str(tmp_path / "j.jsonl")
    j = AllocJournal(path)
    ids = [f"GPU-0-_-{i}" for i in range(5)]
    req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=ids)])
    resp = api.AllocateResponse()
    resp.container_responses.add(envs={const.ENV_RESOURCE_INDEX: "1"})
    body = resp.SerializeToString()
    j.record_fast("uid-a", "default", "a", AllocJournal.fast_head("uid-a", "default", "a", body),
                  req.SerializeToString())
    j2 = AllocJournal(path)                                  # no close(): killed
    assert [e["uid"] for e in j2.unlanded()] == ["uid-a"]
    shuffled = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=ids[::-1])])
    uid, got = j2.lookup(shuffled)
    assert uid == "uid-a" and got().container_responses[0].envs[const.ENV_RESOURCE_INDEX] == "1"
    assert j2.maybe_replay(ids[3])
