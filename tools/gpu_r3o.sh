# Jumbo: the interleaved segment kernel against its own loads (no CRC work) and the LDS-DMA stream;
# the coverage bands (2000 B, 3200 B): segment kernel forced vs the generic kernel.
set -o pipefail
out=gpurun_out/r3o; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab.py --len 9000 --frames 16777216 --rounds 3 --what fcs,dma nstack_amd/libnstack_fcs.so tools/variants/libfcs_segnocrc.so > $out/ab9000.log 2>&1; rc=$?
echo "ab9000 rc=$rc"; grep -v amdgpu.ids $out/ab9000.log | tail -4; [ $rc -ne 0 ] && exit $rc
for L in 2000 3200 1600 2285; do
timeout -k 10 300 python tools/ab.py --len $L --frames $((25000000000 / L)) --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_segany.so > $out/ab$L.log 2>&1; rc=$?
echo "ab$L rc=$rc"; grep -v amdgpu.ids $out/ab$L.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
exit 0
