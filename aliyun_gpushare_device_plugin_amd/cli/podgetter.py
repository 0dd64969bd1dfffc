"""``podgetter`` — dump the kubelet's ``/pods`` (component C15, ``cmd/podgetter/main.go``)."""
from __future__ import annotations

import argparse
import json
import sys

from ..cluster.kubelet import KubeletClient


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="podgetter")
    ap.add_argument("--kubelet-address", default="127.0.0.1")
    ap.add_argument("--kubelet-port", type=int, default=10250)
    ap.add_argument("--token", default="")
    ap.add_argument("--client-cert", default="")
    ap.add_argument("--client-key", default="")
    ap.add_argument("--scheme", default="https")
    a = ap.parse_args(argv)
    kc = KubeletClient.from_flags(a.kubelet_address, a.kubelet_port, a.client_cert, a.client_key, a.token,
                                  scheme=a.scheme)
    pods = kc.get_node_running_pods()
    for p in pods:
        md = p.get("metadata", {})
        print(f"{md.get('namespace')}/{md.get('name')}\t{(p.get('status') or {}).get('phase')}")
    json.dump({"items": len(pods)}, sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
