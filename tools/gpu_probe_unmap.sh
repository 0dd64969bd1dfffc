# one hipMemUnmap over several mappings vs one per mapping (PyTorch's HIP runtime)
set -o pipefail
D=gpurun_out/unmap
mkdir -p $D
timeout -k 10 120 python tools/diag/vmm_unmap_probe.py 16 > $D/unmap16.json 2> $D/unmap16.err
rc=$?; echo "unmap16 rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/diag/vmm_unmap_probe.py 64 > $D/unmap64.json 2> $D/unmap64.err
echo "unmap64 rc=$?" >> $D/steps.log
