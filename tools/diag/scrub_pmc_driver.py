"""A broker scrub to profile: GPU 0's broker (32 GiB) lends its granules to one taker, which hands
them back; the broker zeroes all 32 GiB. Run under rocprofv3 (the broker inherits its tool):

    rocprofv3 --pmc TCC_EA0_WRITE_REQ_64B_sum -d out -o scrub -- python tools/diag/scrub_pmc_driver.py
"""
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from aliyun_gpushare_device_plugin_amd.quota.hbmbroker import HBMBroker  # noqa: E402

d = tempfile.mkdtemp(prefix="gs-scrub-")
b = HBMBroker(os.path.join(d, "hbm.sock"), device=0, gib=32, wait_s=20)
b.start()
try:
    tok = "s" * 32
    b.grant(tok, 32 << 30)
    for _ in range(3):
        c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        c.connect(b.socket_path)
        c.sendall(f"TAKE {tok}\n".encode())
        msg, anc, _, _ = c.recvmsg(4096, socket.CMSG_SPACE(4 * 64))
        fds = [int.from_bytes(x[2][i:i + 4], "little") for x in anc for i in range(0, len(x[2]), 4)]
        for f in fds:
            os.close(f)
        c.close()                                    # handed back: the broker zeroes the granules
        t0 = time.time()
        st = b.stat()
        while (st["free"] < st["granules"] or st["scrubbing"] or st["quarantined"]) and time.time() - t0 < 30:
            time.sleep(0.01)
            st = b.stat()
        print(json.dumps({"scrub_ms_last": st.get("scrub_ms_last"), "scrubbed_bytes": st.get("scrubbed_bytes"),
                          "header": msg.decode(errors="replace").strip()[:60], "fds": len(fds)}), flush=True)
finally:
    b.stop()
