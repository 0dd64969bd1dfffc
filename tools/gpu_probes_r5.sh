# Round-5 hardware probes of the HIP VMM and dma-buf behaviour the HBM broker path depends on
# (results in profiles/r5/): VMM semantics on both runtimes, driver pages next to imported
# granules, and who holds an imported granule's references (system HIP 7.2 and PyTorch's 7.0,
# cold and warm). Each step is bounded; a failing step ends the script.
#   bash tools/gpu_probes_r5.sh <gpurun_out subdir>
set -o pipefail
D=gpurun_out/${1:-probes}
mkdir -p $D
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $D/steps.log; [ $rc -eq 0 ] || exit $rc; }
step vmm_sys timeout -k 10 120 ./tools/diag/build/vmm_semantics_probe 1024 > $D/vmm_semantics_sys.json 2> $D/vmm_semantics_sys.err
step vmm_torch timeout -k 10 180 python tools/diag/vmm_semantics_probe.py 1024 > $D/vmm_semantics_torch.json 2> $D/vmm_semantics_torch.err
step spill timeout -k 10 90 ./tools/diag/build/vmm_spill_probe > $D/vmm_spill.json 2> $D/vmm_spill.err
for w in 0 1 3; do
  step dmabuf_sys_w$w timeout -k 10 90 ./tools/diag/build/dmabuf_ref_probe $w > $D/dmabuf_sys_w$w.json 2> $D/dmabuf_sys_w$w.err
  step dmabuf_torch_w$w timeout -k 10 120 env LD_PRELOAD=$PWD/tools/diag/build/libdmabuf_ref_probe.so python tools/diag/dmabuf_ref_probe.py $w > $D/dmabuf_torch_w$w.json 2> $D/dmabuf_torch_w$w.err
done
