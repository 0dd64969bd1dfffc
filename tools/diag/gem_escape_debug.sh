#!/bin/bash
# Runs the GEM-escape child script of tests/test_gpu_native.py directly, with faulthandler,
# under the quota shim (diagnosis of a crash in that test).
set -o pipefail
cd "$(dirname "$0")/../.."
python -c "import tests.test_gpu_native as t; open('/tmp/gem_escapes.py','w').write(t._GEM_ESCAPES)"
MINOR=$(python -c "from aliyun_gpushare_device_plugin_amd.device import smi as S
with S.SMI('auto') as s: print(s.device(0).render_minor)")
LD_PRELOAD=$PWD/aliyun_gpushare_device_plugin_amd/_native/libgpushare_hipquota.so GPUSHARE_QUOTA_BYTES=$((4<<30)) \
  GPUSHARE_SHIM_LOG=2 timeout -k 5 60 python -X faulthandler /tmp/gem_escapes.py "$MINOR"
