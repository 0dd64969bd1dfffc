"""Drive tools/diag/vmm_broker_probe (build it first with the
hipcc line below). Starts the broker, then tenants one after another, each a fresh process, and
prints one JSON line with every record. This script never touches the GPU itself.

    hipcc --offload-arch=gfx950 -O2 -o tools/diag/build/vmm_broker_probe tools/diag/vmm_broker_probe.cpp
    python tools/diag/vmm_broker_probe.py --granules 48 --granule-mib 1024 --tenants 3
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "vmm_broker_probe")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--granules", type=int, default=48)
    ap.add_argument("--granule-mib", type=int, default=1024)
    ap.add_argument("--tenants", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--tenant-env", action="append", default=[], metavar="K=V",
                    help="extra env of the tenant processes (e.g. LD_PRELOAD of the quota shim)")
    a = ap.parse_args(argv)
    sock = os.path.join(tempfile.mkdtemp(prefix="vmmbroker"), "b.sock")
    br = subprocess.Popen([BIN, "broker", sock, str(a.granules), str(a.granule_mib), str(a.tenants)],
                          stdout=subprocess.PIPE, text=True)
    out = {"granules": a.granules, "granule_mib": a.granule_mib, "tenants": []}
    try:
        first = json.loads(br.stdout.readline() or "{}")
        out["broker"] = first
        if not first.get("broker_ready"):
            print(json.dumps(out), flush=True)
            return 1
        for _ in range(a.tenants):
            tenv = dict(os.environ, **dict(kv.split("=", 1) for kv in a.tenant_env))
            t = subprocess.run([BIN, "tenant", sock], capture_output=True, text=True, timeout=a.timeout, env=tenv)
            rec = json.loads(t.stdout.strip().splitlines()[-1]) if t.stdout.strip() else {}
            rec["rc"] = t.returncode
            if t.returncode:
                rec["stderr"] = t.stderr[-2000:]
            rec["broker"] = json.loads(br.stdout.readline() or "{}")
            out["tenants"].append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
            if t.returncode:
                break
        br.wait(timeout=a.timeout)
        out["broker_rc"] = br.returncode
    finally:
        if br.poll() is None:
            br.kill()
            br.wait()
    print(json.dumps(out), flush=True)
    return 0 if all(r["rc"] == 0 for r in out["tenants"]) and out.get("broker_rc") == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
