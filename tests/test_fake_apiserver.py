"""The fake apiserver's REST/watch semantics (the fidelity the CPU end-to-end tests rest on)."""
import threading
import time

import pytest

from aliyun_gpushare_device_plugin_amd.cluster.client import APIClient, APIError, KubeConfig
from aliyun_gpushare_device_plugin_amd.cluster.podcache import WatchCache
from aliyun_gpushare_device_plugin_amd.sim.apiserver import FakeAPIServer, make_node, strategic_merge
from aliyun_gpushare_device_plugin_amd.sim.cluster import pod_spec


@pytest.fixture()
def api():
    with FakeAPIServer() as s:
        yield s, APIClient(KubeConfig(s.url))


def test_strategic_merge_subset():
    assert strategic_merge({"a": {"b": 1, "c": 2}, "l": [1]}, {"a": {"b": None, "d": 3}, "l": [2]}) == \
        {"a": {"c": 2, "d": 3}, "l": [2]}


def test_crud_selectors_and_binding(api):
    s, c = api
    c.create_node(make_node("n1"))
    c.create_pod("default", pod_spec("a", 2))
    c.create_pod("kube-system", pod_spec("b", 1))
    c.bind_pod("default", "a", "n1")
    items, rv = c.list_pods(field_selector="spec.nodeName=n1,status.phase=Pending")
    assert [p["metadata"]["name"] for p in items] == ["a"] and int(rv) > 0
    assert len(c.list_pods()[0]) == 2 and len(c.list_pods("kube-system")[0]) == 1
    assert len(c.list_pods(field_selector="spec.nodeName!=n1")[0]) == 1
    with pytest.raises(APIError) as e:
        c.bind_pod("default", "a", "n1")
    assert e.value.conflict
    with pytest.raises(APIError) as e:
        c.get_pod("default", "zzz")
    assert e.value.not_found


def test_optimistic_conflict_by_status(api):
    s, c = api
    p = c.create_pod("default", pod_spec("a", 2))
    c.patch_pod("default", "a", {"metadata": {"labels": {"x": "1"}}})
    with pytest.raises(APIError) as e:
        c.patch_pod("default", "a", {"metadata": {"resourceVersion": p["metadata"]["resourceVersion"],
                                                  "labels": {"x": "2"}}})
    assert e.value.conflict and "object has been modified" in e.value.message


def test_node_status_patch_only_touches_status(api):
    s, c = api
    c.create_node(make_node("n1"))
    c.patch_node_status("n1", {"status": {"capacity": {"x": "1"}}, "metadata": {"labels": {"evil": "1"}}})
    n = c.get_node("n1")
    assert n["status"]["capacity"]["x"] == "1" and "evil" not in n["metadata"]["labels"]


def test_watch_replay_and_deleted_on_selector_exit(api):
    s, c = api
    c.create_node(make_node("n1"))
    c.create_pod("default", pod_spec("a", 1))
    _, rv = c.list_pods()
    events, stop = [], threading.Event()

    def run():
        for ev in c.watch_pods("spec.nodeName=n1", rv, 5, stop):
            events.append((ev["type"], ev["object"]["metadata"]["name"]))
    t = threading.Thread(target=run, daemon=True)
    t.start()
    time.sleep(0.2)
    c.bind_pod("default", "a", "n1")                   # enters the selector -> ADDED
    c.patch_pod("default", "a", {"metadata": {"labels": {"k": "v"}}})  # MODIFIED
    c.delete_pod("default", "a")                       # DELETED
    deadline = time.time() + 5
    while len(events) < 3 and time.time() < deadline:
        time.sleep(0.02)
    stop.set()
    assert events == [("ADDED", "a"), ("MODIFIED", "a"), ("DELETED", "a")]


def test_watch_cache_tracks_node_pods(api):
    s, c = api
    c.create_node(make_node("n1"))
    wc = WatchCache(APIClient(KubeConfig(s.url)), "n1").start()
    assert wc.wait_synced(5)
    c.create_pod("default", pod_spec("a", 1))
    c.bind_pod("default", "a", "n1")
    deadline = time.time() + 5
    while not wc.pending_pods() and time.time() < deadline:
        time.sleep(0.02)
    assert [p["metadata"]["name"] for p in wc.pending_pods()] == ["a"]
    c.delete_pod("default", "a")
    while wc.pending_pods() and time.time() < deadline:
        time.sleep(0.02)
    assert wc.pending_pods() == []
    wc.stop()


def test_expired_resource_version_gives_410(api):
    s, c = api
    s.store.history = type(s.store.history)(maxlen=2)
    for i in range(5):
        c.create_pod("default", pod_spec(f"p{i}", 1))
    with pytest.raises(APIError) as e:
        list(c.watch_pods(None, "2", 1))
    assert e.value.gone


def test_service_account_token_rotation(tmp_path, monkeypatch):
    """Round-1 review: the in-cluster token was read once. Now it is re-read on a 401 (one
    retry) and on a timer, for plain requests and for the pod informer's watch."""
    tok = tmp_path / "token"
    tok.write_text("t1\n")
    with FakeAPIServer() as s:
        s.store.valid_tokens = {"t1"}
        cfg = KubeConfig(s.url, token_file=str(tok))
        c = APIClient(cfg)
        c.create_node(make_node("n1"))
        # rotation: the apiserver only accepts the new token; the next call reloads and retries
        tok.write_text("t2\n")
        s.store.valid_tokens = {"t2"}
        assert c.get_node("n1")["metadata"]["name"] == "n1"
        assert cfg.token == "t2" and cfg.token_reloads == 2 and s.store.requests["401"] == 1
        # timer: re-read without waiting for a 401
        monkeypatch.setattr(KubeConfig, "TOKEN_RELOAD_S", 0.0)
        tok.write_text("t3\n")
        s.store.valid_tokens = {"t2", "t3"}
        c.get_node("n1")
        assert cfg.token == "t3" and s.store.requests["401"] == 1
        # a static token (no file) that the apiserver rejects surfaces as 401
        bad = APIClient(KubeConfig(s.url, token="nope"))
        with pytest.raises(APIError) as e:
            bad.get_node("n1")
        assert e.value.status == 401
        # the informer's watch survives a rotation
        monkeypatch.setattr(KubeConfig, "TOKEN_RELOAD_S", 3600.0)
        wc = WatchCache(APIClient(cfg), "n1").start()
        assert wc.wait_synced(5)
        tok.write_text("t4\n")
        s.store.valid_tokens = {"t4"}
        wc.stop()
        wc2 = WatchCache(APIClient(cfg), "n1").start()
        assert wc2.wait_synced(5) and cfg.token == "t4"
        wc2.stop()


def test_kubelet_client_token_reload(tmp_path):
    from aliyun_gpushare_device_plugin_amd.cluster.kubelet import KubeletClient
    from aliyun_gpushare_device_plugin_amd.sim.kubelet import FakeKubelet

    tok = tmp_path / "token"
    tok.write_text("k1")
    with FakeAPIServer() as s:
        kl = FakeKubelet(str(tmp_path / "dp"), APIClient(KubeConfig(s.url)), "n1")
        port = kl.serve_pods(token="k1")
        c = KubeletClient("127.0.0.1", port, token="k1", scheme="http", token_file=str(tok))
        assert c.get_node_running_pods() == []
        tok.write_text("k2")
        kl.pods_token = "k2"
        assert c.get_node_running_pods() == [] and c.token == "k2"
        kl.stop()
