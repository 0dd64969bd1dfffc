"""The deployable scheduler extender (``extender/``): joint placement of the pending queue,
and a restart that rebuilds the ledger from pod annotations (round-3 review item 8)."""
import time

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cluster import objects as O
from aliyun_gpushare_device_plugin_amd.extender import Extender
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster


def test_a_pod_left_out_of_the_joint_plan_does_not_take_planned_room():
    """Queue 16, 64, 128, 128, 128 GiB onto one 288 GiB GPU: the joint plan holds 16+128+128.
    The 64 GiB pod, left out of the plan, must not be placed into the room the plan keeps for
    the second 128 GiB pod (best fit would, stranding 80 GiB)."""
    with SimCluster([("n", "fake:1x288G")]) as c:
        pods = [c.create_pod(s) for s in (16, 64, 128, 128, 128)]
        placed = [c.schedule(p) for p in pods]
        got = [s for s, w in zip((16, 64, 128, 128, 128), placed) if w is not None]
        assert sorted(got) == [16, 128, 128] and sum(got) == 272


def test_restarted_extender_rebuilds_the_ledger_and_never_overcommits():
    """A swapped admission (no admission identity) is rewritten by placement truth; A is deleted;
    the extender restarts with pods still queued. The new instance's ledger comes from the
    annotations alone, so it frees the GPU A really used and places the queue without putting
    more on any GPU than it physically has."""
    with SimCluster([("n", "fake:2x8G")], admission_identity=False) as c:
        c.extender.watch()
        pa, pb = c.create_pod(6, name="a"), c.create_pod(6, name="b")
        assert c.schedule(pa)[1] == 0 and c.schedule(pb)[1] == 1
        adm_b, adm_a = c.admit(pb), c.admit(pa)
        gpu = {"a": int(adm_a.responses[0].envs[const.ENV_RESOURCE_INDEX]),
               "b": int(adm_b.responses[0].envs[const.ENV_RESOURCE_INDEX])}
        assert gpu == {"a": 1, "b": 0}                        # swapped
        m = c.manager("n")
        assert m.allocator.flush_patches(10)
        for name in ("a", "b"):                               # placement truth rewrote both
            got = c.wait_assigned({"metadata": {"namespace": "default", "name": name}})
            assert O.annotations(got)[const.ENV_RESOURCE_INDEX] == str(gpu[name])
        c.delete_pod(c.client.get_pod("default", "a"))        # frees GPU 1 (where A really ran)
        queued = [c.create_pod(8, name="c"), c.create_pod(2, name="d")]   # still pending...
        c.extender.stop_watch()                               # ...when the extender restarts
        ext = Extender(c.client)
        ext.sync()
        for p in queued:
            ext.note_pending(p)                               # its pod informer's initial list
        t = time.monotonic() + 10
        while ext.usage()["n"]["used"] != [6, 0] and time.monotonic() < t:
            time.sleep(0.05)
            ext.sync()
        assert ext.usage()["n"]["used"] == [6, 0]             # B on GPU 0, nothing else
        c.extender = ext
        where = {O.name(p): c.schedule(p) for p in queued}
        assert where["c"] is not None and where["c"][1] == 1  # the 8 GiB pod: only GPU 1 has room
        assert where["d"] is not None and where["d"][1] == 0
        # physical use per GPU (what each admitted container was really given) within capacity
        phys = {0: 6, 1: 0}
        for p in queued:
            adm = c.admit(c.client.get_pod("default", O.name(p)))
            assert adm.error is None
            g = int(adm.responses[0].envs[const.ENV_RESOURCE_INDEX])
            phys[g] += O.gpu_mem_of_pod(p)
        assert phys == {0: 8, 1: 8}
