# Stream kernel v4 vs the flat kernel on homogeneous packed batches (1518 / 576 / 64 B), and the
# fixed-length DMA kernel on 1518 B, to separate the stream's structure from IMIX's mix.
set -o pipefail
out=gpurun_out/r3m; mkdir -p $out; export TMPDIR=/tmp
for m in 1518:1 576:1 64:1; do
  timeout -k 10 300 python tools/ab.py --imix --mix $m --frames 67108864 --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_nostream.so > $out/ab_$m.log 2>&1; rc=$?
  echo "ab $m rc=$rc"; grep -v amdgpu.ids $out/ab_$m.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/ab.py --frames 67108864 --rounds 3 --what fcs,dma nstack_amd/libnstack_fcs.so > $out/ab_fixed.log 2>&1; rc=$?
echo "ab fixed rc=$rc"; grep -v amdgpu.ids $out/ab_fixed.log | tail -3; exit $rc
