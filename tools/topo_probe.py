"""What a GPU box's SMI backends report about the node's GPUs and their links, and the verdict
``bench.py`` would give that topology (``parallel/topology.py``). On a 1-GPU slice of a UBB the
KFD topology in sysfs may still list every GPU of the host; this shows what each backend makes
of it, one JSON line per backend, then the raw KFD io_links of every GPU node.

    python tools/topo_probe.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aliyun_gpushare_device_plugin_amd.device.smi import SMI, SMIError  # noqa: E402
from aliyun_gpushare_device_plugin_amd.parallel import topology as T  # noqa: E402

KFD = "/sys/class/kfd/kfd/topology/nodes"


def kfd_links() -> list:
    out = []
    try:
        nodes = sorted(os.listdir(KFD), key=int)
    except OSError as e:
        return [{"error": str(e)}]
    for n in nodes:
        base = f"{KFD}/{n}"
        try:
            gpu_id = int(open(f"{base}/gpu_id").read().strip() or 0)
        except (OSError, ValueError):
            gpu_id = 0
        links = []
        try:
            for ln in sorted(os.listdir(f"{base}/io_links"), key=int):
                kv = dict(line.split() for line in open(f"{base}/io_links/{ln}/properties") if len(line.split()) == 2)
                links.append({k: kv.get(k) for k in ("type", "node_to", "weight", "max_bandwidth")})
        except OSError:
            pass
        out.append({"node": int(n), "gpu_id": gpu_id, "io_links": links})
    return out


def main():
    for spec in ("auto", "amdsmi", "rocm_smi", "sysfs"):
        row = {"spec": spec}
        try:
            with SMI(spec) as s:
                row["backend"] = s.backend
                n = s.count()
                row["count"] = n
                row["inaccessible"] = s.inaccessible()
                if n:
                    topo = T.build_topology(s)
                    row["link_type"] = topo["link_type"]
                    row["hops"] = topo["hops"]
                    ok, why = T.verdict(topo, n)
                    row["verdict"] = "pass" if ok else "fail"
                    row["reasons"] = why[:8]
        except SMIError as e:
            row["error"] = str(e)
        print(json.dumps(row), flush=True)
    print(json.dumps({"kfd_nodes": kfd_links()}), flush=True)


if __name__ == "__main__":
    main()
