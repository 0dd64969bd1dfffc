#!/bin/bash
# Probe: does the GPU box's kernel expose the dmem cgroup controller (device-memory limits) and does
# amdgpu register its VRAM as a dmem region? Read-only.
set -o pipefail
O=gpurun_out/dmem
mkdir -p $O
{
  echo "uname: $(uname -r)"
  echo "--- mounts (cgroup)"; grep cgroup /proc/mounts
  echo "--- /proc/self/cgroup"; cat /proc/self/cgroup
  for d in /sys/fs/cgroup /sys/fs/cgroup/unified; do
    echo "--- $d"; ls $d 2>&1 | head -80
    echo "controllers: $(cat $d/cgroup.controllers 2>&1)"
    echo "dmem.capacity:"; cat $d/dmem.capacity 2>&1
  done
  echo "--- own cgroup dir"; CG=$(sed -n 's/^0:://p' /proc/self/cgroup); echo "$CG"; ls /sys/fs/cgroup$CG 2>&1 | head -60
  cat /sys/fs/cgroup$CG/dmem.max 2>&1; cat /sys/fs/cgroup$CG/dmem.current 2>&1
  echo "--- kernel config"; (zcat /proc/config.gz 2>/dev/null || cat /boot/config-$(uname -r) 2>/dev/null) | grep -i "DMEM\|CGROUP_DRM" 
  echo "--- amdgpu params"; ls /sys/module/amdgpu/parameters 2>&1 | tr '\n' ' '
} > $O/probe.txt 2>&1
echo done
