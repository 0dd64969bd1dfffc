import os, sys, time, tempfile, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, ROOT)
import test_allocate_engine as T
from aliyun_gpushare_device_plugin_amd.quota import hbmbroker
tmp = tempfile.mkdtemp()
model = T.DeviceModel([T.gpu(i, 288 << 30) for i in range(2)], T.const.GIB)
src = T.StaticSource([])
hdir = os.path.join(tmp, "hbm"); os.mkdir(hdir)
admin = T._FakeBrokerAdmin(hbmbroker.admin_socket(hdir, 1))
opts = T.AllocatorOptions(shim=T.ShimConfig(host_dir=os.path.join(tmp, "shim")), hbm_broker_dir=hdir,
                          ledger_dir=os.path.join(tmp, "ledgers"))
al = T.Allocator(model, src, T.FakeClient(src), T.NODE, opts)
time.sleep(0.5)
def tm(f, n=300):
    xs=[]
    for i in range(n):
        t=time.perf_counter(); f(i); xs.append((time.perf_counter()-t)*1e6)
    return round(statistics.median(xs),1), round(max(xs),1)
pods=[T.mkpod(f"p{i}", 16, 1, 10) for i in range(2000)]
print("prepared", tm(lambda i: al._prepared(pods[i], f"uid-{i}", 1, 16)))
print("ledger take", tm(lambda i: al._ledgers.take(f"uidL-{i}") if al._ledgers else None))
print("token", tm(lambda i: al._hbm.token(f"uidT-{i}", 0)))
print("submit", tm(lambda i: al._hbm.submit(1, al._hbm.token(f"uidS-{i}",0), 16<<30)))
al._hbm._wake.set = lambda: None
print("prepared nowake", tm(lambda i: al._prepared(pods[1000+i], f"uidX-{i}", 1, 16)))
