# Headline: per-workgroup contiguous item ranges (static) vs the product's per-wave dynamic chunks,
# with and without the CRC work (the LDS-DMA read stream), one process.
set -o pipefail
out=gpurun_out/r3r; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab.py --rounds 4 --what fcs,dma nstack_amd/libnstack_fcs.so tools/variants/libfcs_wgstatic.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
