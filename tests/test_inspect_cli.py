"""kubectl-inspect-gpushare (component C14): output format parity with the reference tables."""
import json

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cli import inspect as I
from aliyun_gpushare_device_plugin_amd.utils.tabwriter import format_tabs
from tests.test_allocate_engine import mkpod


def node(name, count, mem, ip="10.0.0.1", ann=None):
    return {"metadata": {"name": name, "annotations": ann or {}},
            "status": {"allocatable": {const.RESOURCE_COUNT: str(count), const.RESOURCE_NAME: str(mem)},
                       "addresses": [{"type": "InternalIP", "address": ip}]}}


def test_tabwriter_matches_go_semantics():
    # Go: cells padded to max width + 2 within a column block; trailing cell unpadded
    assert format_tabs("a\tbb\tc\nccc\td\te\n") == "a    bb  c\nccc  d   e\n"
    # a line without tabs ends the column block
    assert format_tabs("aa\tb\n-----\nc\td\n") == "aa  b\n-----\nc  d\n"


def test_summary_table():
    n = node("n1", 2, 576)
    pods = [mkpod("p1", 64, 0, 1, node="n1", phase="Running"), mkpod("p2", 32, 1, 1, node="n1", phase="Running"),
            mkpod("p3", 16, None, 1, node="n1")]                                  # no index -> pending
    infos = I.build_node_infos(pods, [n])
    assert I.guess_unit(infos) == "GiB"         # 288 units/GPU is an MI355X in GiB (the reference said MiB)
    out = I.display_summary(infos, "GiB")
    lines = out.splitlines()
    assert lines[0].split() == ["NAME", "IPADDRESS", "GPU0(Allocated/Total)", "GPU1(Allocated/Total)",
                                "PENDING(Allocated)", "GPU", "Memory(GiB)"]
    assert lines[1].split() == ["n1", "10.0.0.1", "64/288", "32/288", "16", "112/576"]
    assert set(lines[2]) == {"-"}
    assert lines[3] == "Allocated/Total GPU Memory In Cluster:"
    assert lines[4].strip() == "112/576 (19%)"


def test_unit_from_plugin_annotation_then_heuristic():
    """Round-1 review: the plugin's exported unit wins; without it the fallback threshold
    (1024) keeps an MI355X in GiB (288/GPU) and a 16 GiB card in MiB (16384/GPU)."""
    mib_node = node("m", 1, 288, ann={const.NODE_ANNOTATION_MEMORY_UNIT: "MiB"})   # a 288 MiB slice in MiB mode
    assert I.guess_unit(I.build_node_infos([], [mib_node])) == "MiB"
    assert I.guess_unit(I.build_node_infos([], [node("g", 8, 8 * 288)])) == "GiB"
    assert I.guess_unit(I.build_node_infos([], [node("old", 2, 2 * 16384)])) == "MiB"
    assert I.guess_unit(I.build_node_infos([], [node("x", 0, 0)])) == ""


def test_details_table_and_allocation_annotation():
    n = node("n1", 2, 8)
    p = mkpod("multi", 3, None, 1, node="n1", phase="Running")
    p["metadata"]["annotations"][const.GPUSHARE_ALLOCATION_FLAG] = json.dumps({"0": {"0": 1, "1": 2}})
    q = mkpod("single", 2, 1, 1, node="n1", phase="Running")
    out = I.display_details(I.build_node_infos([p, q], [n]))
    assert "NAME:       n1" in out and "IPADDRESS:  10.0.0.1" in out   # one Go column block
    rows = {ln.split()[0]: ln.split() for ln in out.splitlines() if ln.startswith(("multi", "single"))}
    assert rows["multi"][2:] == ["1", "2"] and rows["single"][2:] == ["0", "2"]
    assert "Allocated :  5 (62%)" in out
    assert out.rstrip().endswith("5/8 (62%)")


def test_terminated_pods_are_ignored():
    pods = [mkpod("done", 4, 0, 1, node="n1", phase="Succeeded"), mkpod("run", 4, 0, 1, node="n1", phase="Running")]
    infos = I.build_node_infos(I.active_pods(pods), [node("n1", 1, 8)])
    assert infos[0].devs[0].used == 4


def test_render_against_live_fake_cluster():
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster
    with SimCluster([("node-a", "fake:2x4G")]) as c:
        c.run_pod(3)
        c.run_pod(2)
        out = I.render(c.client)
        assert "node-a" in out and "5/8" in out and "GPU Memory(GiB)" in out
        assert c.client.get_node("node-a")["metadata"]["annotations"][const.NODE_ANNOTATION_MEMORY_UNIT] == "GiB"
        assert I.render(c.client, "node-a", details=True).count("pod-") == 2
        topo = I.render(c.client, topology=True)
        assert "XGMI1" in topo and "Healthy" in topo
        assert I.main(["--apiserver", c.api_url]) == 0


def test_topology_view_lists_cu_slots():
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster
    with SimCluster([("node-a", "fake:1x309220868096B")], compute_isolation="cu") as c:
        pa, _, _ = c.run_pod(128, name="big")
        pb, _, _ = c.run_pod(64, name="small")
        c.wait_assigned(pa)
        c.wait_assigned(pb)
        topo = I.render(c.client, topology=True)
        assert "CU SLOTS" in topo
        rows = [line.split() for line in topo.splitlines() if line.startswith("GPU0 ") and "-" in line]
        assert ["GPU0", "0-13", "big"] in rows and ["GPU0", "14-20", "small"] in rows
        assert "CU SLOTS" not in I.render(c.client, topology=False)


def test_podgetter_lists_the_kubelets_pods(capsys):
    """``podgetter`` (C15, ``cmd/podgetter/main.go``): the kubelet's /pods, one line per pod."""
    from aliyun_gpushare_device_plugin_amd.cli import podgetter
    from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster

    with SimCluster([("n", "fake:1x8G")]) as c:
        pod, where, adm = c.run_pod(2)
        assert adm.error is None
        kl = c.nodes["n"].kubelet
        port = kl.serve_pods()
        rc = podgetter.main(["--kubelet-address", "127.0.0.1", "--kubelet-port", str(port), "--scheme", "http",
                             "--token", kl.pods_token])
        out, err = capsys.readouterr()
        assert rc == 0 and f"default/{pod['metadata']['name']}\t" in out and '"items": 1' in err
