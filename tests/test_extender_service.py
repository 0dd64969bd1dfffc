"""The deployable scheduler extender (``gpushare-scheduler-extender``, cli/extender.py) as its own
process against the fake apiserver: kube-scheduler's filter and bind calls over HTTP, one pod at
a time, for plain shared pods and for a TP group that must land on an xGMI clique."""
import json
import os
import subprocess
import sys
import time
import urllib.request

from aliyun_gpushare_device_plugin_amd import const
from aliyun_gpushare_device_plugin_amd.cluster import nodestatus, objects as O
from aliyun_gpushare_device_plugin_amd.sim.cluster import SimCluster
from aliyun_gpushare_device_plugin_amd.extender import TP_GROUP_LABEL, TP_SIZE_LABEL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _post(port, verb, body):
    req = urllib.request.Request(f"http://127.0.0.1:{port}/gpushare-scheduler/{verb}", json.dumps(body).encode(),
                                 {"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=10) as r:
        return json.loads(r.read())


def _wait(pred, timeout=10.0):
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if pred():
            return True
        time.sleep(0.02)
    return False


def _schedule(port, c, pod):
    """What kube-scheduler does with the extender: filter over the nodes, bind to the first."""
    nodes = [O.name(n) for n in c.client.list_nodes()]
    f = _post(port, "filter", {"Pod": pod, "NodeNames": nodes})
    if not f["NodeNames"]:
        return None
    b = _post(port, "bind", {"PodName": O.name(pod), "PodNamespace": O.namespace(pod), "PodUID": O.uid(pod),
                             "Node": f["NodeNames"][0]})
    assert b["Error"] == "", b
    return c.client.get_pod(O.namespace(pod), O.name(pod))


def test_extender_process_filter_bind_and_tp_clique():
    with SimCluster([("n", "fake:8x288G")], health_poll_s=0.2) as c:
        env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        proc = subprocess.Popen([sys.executable, "-m", "aliyun_gpushare_device_plugin_amd.cli.extender", "--port", "0",
                                 "--host", "127.0.0.1", "--apiserver", c.api_url, "--resync", "0.5"],
                                env=env, stdout=subprocess.PIPE, text=True)
        try:
            port = int(proc.stdout.readline().split()[1])
            # plain shared pods: best fit, annotations written, the plugin admits them there
            placed = []
            for i in range(6):
                p = _schedule(port, c, c.create_pod(288, name=f"full{i}"))
                assert O.annotations(p)[const.ENV_ASSIGNED_FLAG] == "false"
                placed.append(int(O.annotations(p)[const.ENV_RESOURCE_INDEX]))
                assert c.admit(p).error is None
            assert sorted(placed) == list(range(6))
            # a TP pair with 6<->7 down over xGMI: no node passes the filter
            c.manager("n").smi.inject("linkdown 6 7")
            assert _wait(lambda: nodestatus.read_topology(c.client.get_node("n"))["link_type"][6][7] == "pcie")
            time.sleep(1.0)                                   # the extender's resync picks it up
            labels = {TP_GROUP_LABEL: "g", TP_SIZE_LABEL: "2"}
            a = c.create_pod(64, name="tp-a", labels=labels)
            assert _post(port, "filter", {"Pod": a, "NodeNames": ["n"]})["NodeNames"] == []
            c.manager("n").smi.inject("linkup 6 7")
            assert _wait(lambda: nodestatus.read_topology(c.client.get_node("n"))["link_type"][6][7] == "xgmi")
            time.sleep(1.0)
            b = c.create_pod(64, name="tp-b", labels=labels)
            pa, pb = _schedule(port, c, a), _schedule(port, c, b)
            gpus = sorted(int(O.annotations(p)[const.ENV_RESOURCE_INDEX]) for p in (pa, pb))
            assert gpus == [6, 7]                             # the clique reserved at the first member
            for p in (pa, pb):
                adm = c.admit(p)
                assert adm.error is None
                assert adm.responses[0].envs[const.ENV_RESOURCE_INDEX] == O.annotations(p)[const.ENV_RESOURCE_INDEX]
        finally:
            proc.terminate()
            proc.wait(timeout=10)
