# New segment-kernel selection bounds: segment-kernel parity (all lengths) and the bands in one A/B
# process against the round-2 bound (git HEAD~ build).
set -o pipefail
out=gpurun_out/r3q; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_segil.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
for L in 1950 2000 3073 3200; do
timeout -k 10 300 python tools/ab.py --len $L --frames $((25000000000 / L)) --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_r2bound.so > $out/ab$L.log 2>&1; rc=$?
echo "ab$L rc=$rc"; grep -v amdgpu.ids $out/ab$L.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
exit 0
