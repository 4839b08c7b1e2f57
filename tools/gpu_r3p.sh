# Segment kernel forced vs the generic kernel across the selection bands (one A/B process per length).
set -o pipefail
out=gpurun_out/r3p; mkdir -p $out; export TMPDIR=/tmp
for L in 1525 1560 1700 1800 1900 3049 3100 3300 4573 6100; do
timeout -k 10 300 python tools/ab.py --len $L --frames $((25000000000 / L)) --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_segany.so > $out/ab$L.log 2>&1; rc=$?
echo "ab$L rc=$rc"; grep -v amdgpu.ids $out/ab$L.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
exit 0
