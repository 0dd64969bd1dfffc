"""Property tests (hypothesis) for the invariants the sharing protocol rests on.

* the extender's best-fit ledger never over-commits a GPU, whatever the create/delete order;
* the Allocate engine never hands one pod to two requests and only matches equal sizes,
  oldest assume time first (``allocate.go:63-89``);
* ``best_group`` returns distinct, pairwise one-hop xGMI GPUs that all fit the request;
* unit / quota arithmetic is monotone and never exceeds the real device bytes.
"""
import itertools

from hypothesis import HealthCheck, given, settings, strategies as st

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.parallel import topology as T
from aliyun_gpushare_device_plugin_amd.sim.extender import ExtenderSim, NodeState
from aliyun_gpushare_device_plugin_amd.utils import units as U

from .test_allocate_engine import FakeClient, StaticSource, mkpod
from .test_units_and_model import gpu

FAST = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def _pod(uid, size):
    return {"metadata": {"name": uid, "namespace": "default", "uid": uid, "annotations": {}},
            "spec": {"containers": [{"name": "c", "resources": {"limits": {const.RESOURCE_NAME: str(size)}}}]},
            "status": {"phase": "Pending"}}


@FAST
@given(ngpu=st.integers(1, 8), cap=st.sampled_from([8, 64, 288]),
       ops=st.lists(st.tuples(st.booleans(), st.integers(1, 160)), min_size=1, max_size=80))
def test_extender_never_overcommits(ngpu, cap, ops):
    ext = ExtenderSim(client=None)
    ext.nodes["n"] = NodeState("n", ngpu, cap, [0] * ngpu, None, [True] * ngpu)
    live, seq = [], itertools.count()
    for create, size in ops:
        if create or not live:
            p = _pod(f"p{next(seq)}", size)
            where = ext.decide(p)
            if where is None:
                assert all(cap - u < size for u in ext.nodes["n"].used)
            else:
                live.append((p, size, where[1]))
        else:
            p, _, _ = live.pop(size % len(live))
            ext.forget(p)
        used = ext.nodes["n"].used
        assert all(0 <= u <= cap for u in used)
        assert used == [sum(s for _, s, g in live if g == i) for i in range(ngpu)]


@FAST
@given(sizes=st.lists(st.integers(1, 4), min_size=1, max_size=12), reqs=st.lists(st.integers(1, 4), max_size=16))
def test_allocate_matches_each_pod_once_oldest_first(sizes, reqs):
    pods = [mkpod(f"p{i}", s, i % 2, 1000 + i) for i, s in enumerate(sizes)]
    model = DeviceModel([gpu(0, 4 << 30), gpu(1, 4 << 30)], const.GIB)
    src = StaticSource(pods)
    al = Allocator(model, src, FakeClient(src), "node-a", AllocatorOptions(complete_swaps=False))
    taken, ids = set(), itertools.count()
    for r in reqs:
        req = api.AllocateRequest()     # fresh fake IDs per admission, as the kubelet hands out
        req.container_requests.add().devices_ids.extend([f"GPU-{0:016x}-_-{next(ids)}" for _ in range(r)])
        envs = dict(al.allocate(req).container_responses[0].envs)
        remaining = [p for p in pods if p["metadata"]["name"] not in taken and
                     int(p["spec"]["containers"][0]["resources"]["limits"][const.RESOURCE_NAME]) == r]
        if not remaining:
            assert envs[const.ENV_RESOURCE_INDEX] == "-1"
            continue
        oldest = min(remaining, key=lambda p: int(p["metadata"]["annotations"][const.ENV_RESOURCE_ASSUME_TIME]))
        name = oldest["metadata"]["name"]
        assert envs[const.ENV_RESOURCE_INDEX] == oldest["metadata"]["annotations"][const.ENV_RESOURCE_INDEX]
        assert name not in taken
        taken.add(name)


def _topo(n, links):
    lt = [["self" if i == j else "pcie" for j in range(n)] for i in range(n)]
    hops = [[0 if i == j else 3 for j in range(n)] for i in range(n)]
    for a, b in links:
        if a != b:
            lt[a][b] = lt[b][a] = "xgmi"
            hops[a][b] = hops[b][a] = 1
    return {"link_type": lt, "hops": hops}


@FAST
@given(n=st.integers(2, 8), data=st.data())
def test_best_group_is_xgmi_clique_that_fits(n, data):
    links = data.draw(st.sets(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1)), max_size=n * n))
    free = data.draw(st.lists(st.integers(0, 288), min_size=n, max_size=n))
    size = data.draw(st.integers(1, n))
    req = data.draw(st.integers(1, 288))
    topo = _topo(n, links)
    grp = T.best_group(topo, free, size, req)
    cliques = [c for c in itertools.combinations(range(n), size)
               if all(free[i] >= req for i in c) and all(T.xgmi_connected(topo, a, b)
                                                        for a, b in itertools.combinations(c, 2))]
    if grp is None:
        assert not cliques
    else:
        assert len(set(grp)) == size and tuple(sorted(grp)) in cliques
        # best fit: no other valid group leaves less capacity unused
        assert sum(free[i] - req for i in grp) == min(sum(free[i] - req for i in c) for c in cliques)


@FAST
@given(nbytes=st.integers(1, 1 << 40), extra=st.integers(0, 1 << 30), unit=st.sampled_from([const.GIB, const.MIB]),
       policy=st.sampled_from(["floor", "nearest"]))
def test_units_monotone(nbytes, extra, unit, policy):
    assert U.units_for_bytes(nbytes, unit, policy) <= U.units_for_bytes(nbytes + extra, unit, policy)
    if policy == "floor":
        assert U.units_for_bytes(nbytes, unit, policy) * const.UNIT_BYTES[unit] <= nbytes


@FAST
@given(dev_units=st.integers(1, 300_000), dev_bytes=st.integers(1, 1 << 40), c1=st.integers(0, 300_000),
       c2=st.integers(0, 300_000))
def test_quota_bounded_and_monotone(dev_units, dev_bytes, c1, c2):
    lo, hi = sorted((c1, c2))
    assert 0 <= U.quota_bytes(lo, dev_units, dev_bytes) <= U.quota_bytes(hi, dev_units, dev_bytes) <= dev_bytes
    # co-located containers that fit the device's units never exceed its bytes together
    if lo + hi <= dev_units:
        assert U.quota_bytes(lo, dev_units, dev_bytes) + U.quota_bytes(hi, dev_units, dev_bytes) <= dev_bytes


@FAST
@given(v=st.integers(0, 10 ** 6), suffix=st.sampled_from(["", "k", "M", "Ki", "Mi", "Gi"]))
def test_parse_quantity_scales(v, suffix):
    mult = {"": 1, "k": 10 ** 3, "M": 10 ** 6, "Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30}[suffix]
    assert U.parse_quantity(f"{v}{suffix}") == v * mult
