"""Property tests (hypothesis) for the invariants the sharing protocol rests on.

* the extender's best-fit ledger never over-commits a GPU, whatever the create/delete order;
* the Allocate engine never hands one pod to two requests and only matches equal sizes,
  oldest assume time first (``allocate.go:63-89``);
* ``best_group`` returns distinct, pairwise one-hop xGMI GPUs that all fit the request;
* unit / quota arithmetic is monotone and never exceeds the real device bytes.
"""
import itertools

import pytest

from hypothesis import HealthCheck, given, settings, strategies as st

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api
from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
from aliyun_gpushare_device_plugin_amd.parallel import topology as T
from aliyun_gpushare_device_plugin_amd.extender import Extender, NodeState
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
    ext = Extender(client=None)
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


def _admit_all(pods, order, ngpu, cap, strict=True):
    """Drive the engine like the kubelet: pods one at a time in ``order``, one Allocate per gpu
    container, back to back; a refused container fails the pod's admission (strict mode = the
    kubelet's UnexpectedAdmissionError) and it turns Failed, an admitted pod turns Running."""
    import time as _t

    from aliyun_gpushare_device_plugin_amd.alloc.engine import AllocationError

    model = DeviceModel([gpu(i, cap << 30) for i in range(ngpu)], const.GIB)
    src = StaticSource(pods)
    cl = FakeClient(src)
    al = Allocator(model, src, cl, "node-a", AllocatorOptions(strict=strict))
    ids = itertools.count()
    granted = {}                                   # pod name -> [gpu idx per container]
    for i in order:
        p = pods[i]
        shape = [int(c["resources"]["limits"][const.RESOURCE_NAME]) for c in p["spec"]["containers"]]
        got = []
        for size in shape:
            req = api.AllocateRequest()
            req.container_requests.add().devices_ids.extend([f"id-{next(ids)}" for _ in range(size)])
            try:
                envs = dict(al.allocate(req).container_responses[0].envs)
            except AllocationError:
                got = None
                break
            got.append(int(envs[const.ENV_RESOURCE_INDEX]))
        p["status"]["phase"] = "Running" if got is not None else "Failed"
        granted[p["metadata"]["name"]] = got
        _t.sleep(0)
    return granted, cl


@settings(max_examples=500, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(ngpu=st.integers(1, 4), data=st.data())
def test_admission_orders_keep_reservations_exact(ngpu, data):
    """Round-1 review item: random mixes of single- and multi-container pods, extender-reserved
    on N GPUs, admitted in an arbitrary kubelet order. Invariants:
    * the GPU a container is granted is never over-committed: Σ granted per GPU over admitted
      pods ≤ Σ reserved there ≤ capacity (every grant consumes an equal-size container of some
      reservation, so accounting by pod annotations stays exact);
    * a pod's containers are granted or refused cleanly (strict mode), never a bogus index;
    * no pod is PATCHed ASSIGNED twice;
    * all pods single-container: every pod is admitted, and the granted (size, GPU) multiset
      equals the reserved one (equal-size pods may swap reservations, nothing else);
    * admission in assume-time order: every container gets its own pod's reserved GPU."""
    import time as _t

    cap = 12
    shapes = data.draw(st.lists(st.lists(st.integers(1, 5), min_size=1, max_size=3), min_size=1, max_size=10))
    single = data.draw(st.booleans())
    if single:
        shapes = [s[:1] for s in shapes]
    free = [cap] * ngpu
    pods, reserved = [], []
    now = _t.time_ns()
    for i, shape in enumerate(shapes):
        g = next((j for j in range(ngpu) if free[j] >= sum(shape)), None)   # extender first-fit
        if g is None:
            continue
        free[g] -= sum(shape)
        pods.append(mkpod(f"p{i}", shape, g, now - 10_000 + i))
        reserved.append((tuple(shape), g))
    in_order = data.draw(st.booleans())
    order = list(range(len(pods))) if in_order else data.draw(st.permutations(range(len(pods))))
    granted, cl = _admit_all(pods, order, ngpu, cap)

    names = [p[1] for p in cl.patches]
    assert len(names) == len(set(names))
    used = [0] * ngpu
    for p, (shape, g) in zip(pods, reserved):
        got = granted[p["metadata"]["name"]]
        if got is None:
            continue
        assert all(0 <= x < ngpu for x in got)
        for size, x in zip(shape, got):
            used[x] += size
    reserved_per_gpu = [sum(sum(s) for s, g in reserved if g == j) for j in range(ngpu)]
    assert all(u <= r <= cap for u, r in zip(used, reserved_per_gpu))
    if single:
        assert all(granted[p["metadata"]["name"]] is not None for p in pods)
        got = sorted((s, granted[p["metadata"]["name"]][0]) for p, (s, _) in zip(pods, reserved))
        assert got == sorted(reserved)
    if in_order:
        for p, (shape, g) in zip(pods, reserved):
            assert granted[p["metadata"]["name"]] == [g] * len(shape)


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(nbins=st.integers(1, 8), data=st.data())
def test_joint_packing_is_feasible_and_beats_best_fit(nbins, data):
    """extender/packing.py: the joint plan never over-fills a GPU, is never worse than best fit (in
    arrival order or decreasing), and packs everything when a perfect packing exists (items cut
    from the bins themselves, then shuffled)."""
    from aliyun_gpushare_device_plugin_amd.extender.packing import best_fit, pack

    cap = data.draw(st.sampled_from([64, 288]))
    free = [cap] * nbins
    items = []
    for _ in range(nbins):                      # cut every bin into 1-5 pieces: a perfect packing
        left, cuts = cap, data.draw(st.integers(1, 5))
        for _ in range(cuts - 1):
            piece = data.draw(st.integers(1, max(1, left - 1))) if left > 1 else 0
            if piece <= 0 or piece >= left:
                break
            items.append(piece)
            left -= piece
        items.append(left)
    extra = data.draw(st.lists(st.integers(1, cap), max_size=4))  # over-subscription
    sizes = data.draw(st.permutations(items + extra))
    got = pack(free, sizes, budget=20_000)
    used = [0] * nbins
    for a, s in zip(got, sizes):
        if a is not None:
            used[a] += s
    assert all(u <= cap for u in used)

    def score(x):
        return sum(a is not None for a in x), sum(s for a, s in zip(x, sizes) if a is not None)

    assert score(got) >= score(best_fit(free, sizes, list(range(len(sizes)))))
    assert score(got) >= score(best_fit(free, sizes, sorted(range(len(sizes)), key=lambda k: -sizes[k])))
    if not extra:
        assert score(got)[0] == len(sizes), (free, sizes, got)


@pytest.mark.parametrize("nbins,cap,sizes", [
    (7, 288, [288, 288, 178, 154, 133, 125, 98, 94, 90, 86, 76, 69, 58, 54, 41, 38, 35, 27, 23, 20, 13, 9, 8, 6, 5]),
    (7, 64, [59, 50, 43, 41, 34, 29, 22, 22, 18, 17, 16, 14, 13, 11, 11, 8, 7, 7, 6, 5, 5, 4, 3, 3]),
    (8, 288, [255, 210, 203, 191, 150, 149, 139, 134, 124, 119, 109, 102, 70, 55, 46, 45, 33, 23, 20, 19, 15, 13,
              13, 12, 10, 10, 9, 8, 8, 6, 4]),
])
def test_zero_slack_perfect_packings_are_found(nbins, cap, sizes):
    """Pods that exactly fill every GPU (no slack): item-by-item search missed these within
    200k expansions; bin completion (extender/packing.py place_all) finds them in a few hundred."""
    from aliyun_gpushare_device_plugin_amd.extender.packing import pack, place_all

    assert sum(sizes) == nbins * cap
    for got in (place_all([cap] * nbins, sizes, budget=2_000), pack([cap] * nbins, sizes, budget=4_000)):
        assert got is not None and None not in got
        used = [0] * nbins
        for a, s in zip(got, sizes):
            used[a] += s
        assert used == [cap] * nbins


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(ops=st.lists(st.tuples(st.sampled_from(["add", "add", "add", "run", "delete", "assign", "claim", "taint"]),
                              st.integers(0, 7), st.integers(1, 3), st.integers(0, 1), st.integers(0, 40)),
                    min_size=1, max_size=25))
def test_table_hook_equals_a_full_rebuild(ops):
    """alloc/engine.py ``_publish_change``: after any sequence of pod-cache changes (pods bound,
    admitted, deleted, assigned by a patch) and engine-side changes (claims, taints), the table
    the watch-thread hook published is entry for entry the one a full ``_prepare`` builds."""
    import json as _json
    import time

    from aliyun_gpushare_device_plugin_amd import const as C
    from aliyun_gpushare_device_plugin_amd.alloc.engine import Allocator, AllocatorOptions
    from aliyun_gpushare_device_plugin_amd.cluster.podcache import WatchCache
    from aliyun_gpushare_device_plugin_amd.device.model import DeviceModel
    from tests.test_allocate_engine import FakeClient, mkpod
    from tests.test_units_and_model import gpu

    class Nat:
        spin_us = 0

        def publish(self, blob):
            pass

        def set_version(self, v):
            pass

        def set_gen(self, g):
            pass

    cache = WatchCache(client=None, node="node-a")
    cache._synced.set()
    al = Allocator(DeviceModel([gpu(0, 8 << 30), gpu(1, 8 << 30)], C.GIB), cache, FakeClient(cache), "node-a",
                   AllocatorOptions(async_patch=True, fast_path=False))
    al.native = Nat()
    al.opts.fast_path = True
    cache.on_pending_change = al._on_pending
    al._prepare(cache)
    pods: dict = {}
    rv = [1]

    def put(p, typ="MODIFIED"):
        rv[0] += 1
        p = _json.loads(_json.dumps(p))
        p["metadata"]["resourceVersion"] = str(rv[0])
        cache._apply({"type": typ, "object": p})
        return p

    def expected():
        with al._mu:
            cands = [p for p in al._candidates(fresh=False) if p["metadata"]["uid"] not in al._claims]
        out = []
        for p in cands:
            shape = al._info(p)[3]
            if shape and (len(shape) > 1 or al.model.gpu(int(p["metadata"]["annotations"][C.ENV_RESOURCE_INDEX])) is not None):
                out.append(p["metadata"]["uid"])
        return out

    try:
        for op, k, size, g, at in ops:
            name = f"p{k}"
            cur = pods.get(name)
            if op == "add" and cur is None:
                pods[name] = put(mkpod(name, size, g, 100 + at), "ADDED")
            elif op == "run" and cur is not None:
                cur["status"]["phase"] = "Running"
                pods[name] = put(cur)
            elif op == "delete" and cur is not None:
                put(cur, "DELETED")
                del pods[name]
            elif op == "assign" and cur is not None:
                cur["metadata"]["annotations"][C.ENV_ASSIGNED_FLAG] = "true"
                pods[name] = put(cur)
            elif op == "claim" and cur is not None:
                with al._mu:                                   # a native answer taken in
                    al._assigned[cur["metadata"]["uid"]] = time.monotonic()
            elif op == "taint" and cur is not None:
                with al._mu:
                    al._tainted[cur["metadata"]["uid"]] = time.monotonic()
                    al._bump_gen()
                al._prepare(cache)                             # a generation change: the full path
            v, gen, out, _ = al._last_table
            assert (v, gen) == (cache.pending_version, al._gen)
            got = [c.uid for c in out]
            # claims taken after the table was built stay in it (the server marks them taken)
            want = expected()
            assert [u for u in got if u not in al._assigned] == want, (op, name, got, want)
    finally:
        al.native = None
        al.close()
