#!/bin/bash
# One-shot environment probe of the GPU box (SMI, sysfs, device nodes).
out=gpurun_out/probe
mkdir -p $out
{
echo "== id"; id; echo "== nproc"; nproc
echo "== ls /dev/dri"; ls -la /dev/dri /dev/kfd 2>&1
echo "== kfd nodes"; ls /sys/class/kfd/kfd/topology/nodes/ 2>&1
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "--- $n"; cat $n/properties 2>&1 | head -60; cat $n/name 2>&1; ls $n/io_links 2>&1; ls $n/mem_banks 2>&1; done
echo "== io_links node1"; for l in /sys/class/kfd/kfd/topology/nodes/1/io_links/*; do echo "-- $l"; cat $l/properties; done
echo "== mem bank node1"; for l in /sys/class/kfd/kfd/topology/nodes/1/mem_banks/*; do echo "-- $l"; cat $l/properties; done
echo "== drm"; ls -la /sys/class/drm/ 2>&1
for c in /sys/class/drm/card*; do echo "--- $c"; ls $c/device 2>&1 | head -200; for f in mem_info_vram_total mem_info_vram_used unique_id product_name serial_number current_compute_partition current_memory_partition available_compute_partition numa_node vendor device; do echo "$f=$(cat $c/device/$f 2>&1)"; done; done
echo "== rocm-smi"; timeout 60 rocm-smi 2>&1 | head -40
echo "== rocm-smi showmeminfo"; timeout 60 rocm-smi --showmeminfo vram --showuniqueid --showbus --showtopo --json 2>&1 | head -100
echo "== amd-smi"; timeout 60 amd-smi list 2>&1 | head -40; timeout 60 amd-smi static -g 0 2>&1 | head -80
echo "== amd-smi topology"; timeout 60 amd-smi topology 2>&1 | head -40
echo "== rocminfo"; timeout 60 rocminfo 2>&1 | grep -E 'Name:|Uuid|Marketing|Compute Unit' | head -30
echo "== env"; env | grep -E 'HIP|ROCR|HSA|CUDA|GPU|ROCM' 
echo "== rocprofv3 help"; rocprofv3 --help 2>&1 | grep -iE 'memory|alloc|scratch' | head -20
} > $out/probe.txt 2>&1
python3 - > $out/torch.txt 2>&1 <<'PY'
import torch, time
t=time.time()
print(torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
p=torch.cuda.get_device_properties(0)
print(p)
print("mem_get_info", torch.cuda.mem_get_info())
import ctypes
hip=ctypes.CDLL("libamdhip64.so")
free=ctypes.c_size_t(); tot=ctypes.c_size_t()
print("hipMemGetInfo", hip.hipMemGetInfo(ctypes.byref(free),ctypes.byref(tot)), free.value, tot.value)
# allocation granularity probe via hipMemGetInfo deltas
for sz in [1, 4096, 65536, 2<<20, (2<<20)+1, 64<<20, (64<<20)+4096, 1<<30]:
    f0=ctypes.c_size_t(); t0=ctypes.c_size_t(); hip.hipMemGetInfo(ctypes.byref(f0),ctypes.byref(t0))
    ptr=ctypes.c_void_p()
    rc=hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(sz))
    f1=ctypes.c_size_t(); hip.hipMemGetInfo(ctypes.byref(f1),ctypes.byref(t0))
    print("alloc", sz, "rc", rc, "delta", f0.value-f1.value, "ptr", hex(ptr.value or 0))
    hip.hipFree(ptr)
print("elapsed", time.time()-t)
PY
echo done
