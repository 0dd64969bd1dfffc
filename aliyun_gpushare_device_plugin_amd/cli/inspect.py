"""``kubectl-inspect-gpushare`` — cluster GPU-memory report (component C14).

Reference ``cmd/inspect/{main,podinfo,nodeinfo,display}.go``: per-node, per-GPU usage is
rebuilt from pod specs and annotations only (the plugin is never queried); per-GPU total is
``allocatable[gpu-mem] / allocatable[gpu-count]``; pods carry either the newer
``scheduler.framework.gpushare.allocation`` JSON or the legacy ``ALIYUN_COM_GPU_MEM_IDX``;
pods without an index land in a PENDING column (device -1). The unit comes from the
``gpushare.amd.com/memory-unit`` node annotation the plugin writes; only nodes without it fall
back to a guess from the per-GPU units. The reference's guess (> 100 → MiB,
``nodeinfo.go:228-244``) calls a 288 GiB MI355X "MiB", so the fallback threshold is 1024:
every GPU between 1 GiB and 1 TiB is ≥ 1024 in MiB and < 1024 in GiB. Summary (default) and ``-d`` detail tables keep the reference
layout byte for byte (Go tabwriter emulation). ``--topology`` adds the MI355X xGMI matrix and
per-GPU health exported by the plugin (no reference counterpart).

Fixed: ``getNodes`` dereferenced the node before checking the error.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import sys
import time

from .. import const
from ..alloc import annotations as A
from ..cluster import nodestatus, objects as O
from ..cluster.client import APIClient, APIError, build_client
from ..utils.tabwriter import TabWriter


@dataclasses.dataclass
class DeviceInfo:
    idx: int
    total: int
    used: int = 0
    pods: list = dataclasses.field(default_factory=list)

    def __str__(self):
        return f"{self.used}" if self.idx == -1 else f"{self.used}/{self.total}"


@dataclasses.dataclass
class NodeInfo:
    node: dict
    pods: list
    gpu_count: int
    gpu_total: int
    devs: dict

    @property
    def name(self):
        return O.name(self.node)

    def has_pending(self) -> bool:
        return -1 in self.devs


def gpu_memory_in_pod(pod: dict) -> int:
    return O.gpu_mem_of_pod(pod)


def device_allocation(pod: dict) -> dict[int, int]:
    """``getDeivceInfo`` (``nodeinfo.go:169-197``)."""
    alloc = A.allocation_from_annotation(pod)
    if alloc:
        return alloc
    idx = -1
    v = O.annotations(pod).get(const.ENV_RESOURCE_INDEX)
    if v is not None:
        try:
            idx = int(v)
        except ValueError:
            idx = -1
    return {idx: gpu_memory_in_pod(pod)}


def build_node_infos(pods: list[dict], nodes: list[dict]) -> list[NodeInfo]:
    infos = []
    for node in nodes:
        cnt = O.node_allocatable(node, const.RESOURCE_COUNT)
        tot = O.node_allocatable(node, const.RESOURCE_NAME)
        per = tot // cnt if cnt > 0 else 0
        devs = {i: DeviceInfo(i, per) for i in range(cnt)}
        mine = [p for p in pods if O.node_name(p) == O.name(node)]
        info = NodeInfo(node, mine, cnt, tot, devs)
        if tot > 0:
            for p in mine:
                if gpu_memory_in_pod(p) <= 0:
                    continue
                for dev, used in device_allocation(p).items():
                    d = info.devs.setdefault(dev, DeviceInfo(dev, per))
                    d.used += used
                    d.pods.append(p)
        infos.append(info)
    return infos


MIB_GUESS_THRESHOLD = 1024


def guess_unit(infos: list[NodeInfo]) -> str:
    """``setUnit`` (``nodeinfo.go:228-244``): the first node with GPUs decides — by the unit
    its plugin exported, else by the size heuristic (see the module docstring)."""
    for i in infos:
        u = O.annotations(i.node).get(const.NODE_ANNOTATION_MEMORY_UNIT)
        if i.gpu_total > 0 and u in (const.GIB, const.MIB):
            return u
    for i in infos:
        if i.gpu_total > 0 and i.gpu_count > 0:
            return const.MIB if i.gpu_total // i.gpu_count >= MIB_GUESS_THRESHOLD else const.GIB
    return ""


def display_summary(infos: list[NodeInfo], unit: str) -> str:
    w = TabWriter()
    max_gpu = max((i.gpu_count for i in infos), default=0)
    has_pending = any(i.has_pending() for i in infos)
    hdr = "NAME\tIPADDRESS\t" + "".join(f"GPU{i}(Allocated/Total)\t" for i in range(max_gpu))
    if has_pending:
        hdr += "PENDING(Allocated)\t"
    hdr += f"GPU Memory({unit})\n"
    w.write(hdr)
    used_c = total_c = 0
    line_len = 0
    for info in infos:
        if info.gpu_total <= 0:
            continue
        used_n = 0
        cells = []
        for i in range(max_gpu):
            d = info.devs.get(i)
            if d is not None:
                cells.append(str(d))
                used_n += d.used
            else:
                cells.append("0/0")
        pending = ""
        if -1 in info.devs:
            pending = str(info.devs[-1].used)
            used_n += info.devs[-1].used
        row = f"{info.name}\t{O.node_internal_ip(info.node)}\t" + "".join(c + "\t" for c in cells)
        if has_pending:
            row += pending + "\t"
        row += f"{used_n}/{info.gpu_total}\n"
        w.write(row)
        if line_len == 0:
            line_len = len(row) + 20
        used_c += used_n
        total_c += info.gpu_total
    w.write("-" * line_len + "\n")
    w.write("Allocated/Total GPU Memory In Cluster:\n")
    pct = int(used_c / total_c * 100) if total_c > 0 else 0
    w.write(f"{used_c}/{total_c} ({pct}%)\t\n")
    return w.flush()


def display_details(infos: list[NodeInfo]) -> str:
    w = TabWriter()
    used_c = total_c = 0
    line_len = 0
    for info in infos:
        if info.gpu_total <= 0:
            continue
        w.write("\n")
        w.write(f"NAME:\t{info.name}\n")
        w.write(f"IPADDRESS:\t{O.node_internal_ip(info.node)}\n")
        w.write("\n")
        hdr = "NAME\tNAMESPACE\t" + "".join(f"GPU{i}(Allocated)\t" for i in range(info.gpu_count))
        if info.has_pending():
            hdr += "Pending(Allocated)\t"
        w.write(hdr + "\n")
        rows = []
        seen = set()
        used_n = 0
        for i in sorted(info.devs):
            dev = info.devs[i]
            used_n += dev.used
            for pod in dev.pods:
                if O.uid(pod) in seen:
                    continue
                r = f"{O.name(pod)}\t{O.namespace(pod)}\t"
                count = info.gpu_count + (1 if info.has_pending() else 0)
                alloc = A.allocation_from_annotation(pod)
                for k in range(count):
                    if alloc:
                        r += f"{alloc.get(k, 0)}\t"
                    elif k == i or (i == -1 and k == info.gpu_count):
                        r += f"{gpu_memory_in_pod(pod)}\t"
                    else:
                        r += "0\t"
                rows.append(r + "\n")
                seen.add(O.uid(pod))
        body = "".join(rows)
        if line_len == 0:
            line_len = len(body) + 10
        w.write(body)
        pct = int(used_n / info.gpu_total * 100) if info.gpu_total > 0 else 0
        w.write(f"Allocated :\t{used_n} ({pct}%)\t\n")
        w.write(f"Total :\t{info.gpu_total} \t\n")
        w.write("-" * line_len + "\n")
        total_c += info.gpu_total
        used_c += used_n
    w.write("\n\nAllocated/Total GPU Memory In Cluster:\t")
    pct = int(used_c / total_c * 100) if total_c > 0 else 0
    w.write(f"{used_c}/{total_c} ({pct}%)\t\n")
    return w.flush()


def display_topology(infos: list[NodeInfo]) -> str:
    out = []
    for info in infos:
        topo = nodestatus.read_topology(info.node)
        health = json.loads(O.annotations(info.node).get(const.NODE_ANNOTATION_HEALTH, "{}") or "{}")
        out.append(f"\nNODE {info.name}  hive {topo.get('hive_id') if topo else '-'}")
        if topo:
            n = len(topo["link_type"])
            w = TabWriter()
            w.write("\t" + "".join(f"GPU{j}\t" for j in range(n)) + "HEALTH\n")
            for i in range(n):
                row = f"GPU{i}\t" + "".join(
                    f"{topo['link_type'][i][j].upper()}{topo['hops'][i][j] if i != j else ''}\t" for j in range(n))
                h = health.get(str(i), {})
                row += ("Healthy" if h.get("healthy", True) else f"Unhealthy({h.get('reason', '')})") + "\n"
                w.write(row)
            out.append(w.flush())
        slots = cu_slot_rows(info)
        if slots:
            out.append("CU SLOTS (--compute-isolation=cu; slot s = CU s of every XCD)\n" + slots)
    return "\n".join(out) + "\n"


def cu_slot_rows(info: NodeInfo) -> str:
    """Per GPU: the CU-slot run each active pod holds (``gpushare.amd.com/cu-slots``)."""
    from ..alloc.cuslots import SlotRun

    per: dict[int, list] = {}
    for p in info.pods:
        r = SlotRun.parse(O.annotations(p).get(const.POD_ANNOTATION_CU_SLOTS))
        if r is None:
            continue
        per.setdefault(A.gpu_id_from_annotation(p), []).append((r.start, r, O.name(p)))
    if not per:
        return ""
    w = TabWriter()
    w.write("GPU\tSLOTS\tPOD\n")
    for g in sorted(per):
        for _, r, name in sorted(per[g]):
            w.write(f"GPU{g}\t{r.annotation()}\t{name}\n")
    return w.flush()


def active_pods(pods: list[dict]) -> list[dict]:
    return [p for p in pods if not O.is_terminated(p)]


def list_with_retries(fn, retries=5, sleep=0.1):
    err = None
    for _ in range(retries + 1):
        try:
            return fn()
        except (APIError, OSError) as e:
            err = e
            time.sleep(sleep)
    raise err


def collect(client: APIClient, node_name: str | None):
    if node_name:
        nodes = [client.get_node(node_name)]
        pods, _ = list_with_retries(lambda: client.list_pods(field_selector=f"spec.nodeName={node_name}"))
    else:
        nodes = [n for n in client.list_nodes() if O.node_allocatable(n, const.RESOURCE_NAME) > 0]
        pods, _ = list_with_retries(lambda: client.list_pods())
    return nodes, active_pods(pods)


def render(client: APIClient, node_name: str | None = None, details: bool = False, topology: bool = False) -> str:
    nodes, pods = collect(client, node_name)
    infos = build_node_infos(pods, nodes)
    unit = guess_unit(infos)
    s = display_details(infos) if details else display_summary(infos, unit)
    if topology:
        s += display_topology(infos)
    return s


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kubectl-inspect-gpushare")
    ap.add_argument("-d", action="store_true", help="details")
    ap.add_argument("--topology", action="store_true", help="show xGMI topology and GPU health (MI355X)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--apiserver", default=None)
    ap.add_argument("node", nargs="?", default=None)
    a = ap.parse_args(argv)
    try:
        client = build_client(a.kubeconfig, a.apiserver, timeout=15)
        sys.stdout.write(render(client, a.node, a.d, a.topology))
    except Exception as e:  # noqa: BLE001
        print(f"Failed due to {e}", end="")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
