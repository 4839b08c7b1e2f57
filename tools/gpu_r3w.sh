set -o pipefail
out=gpurun_out/r3w; mkdir -p $out
timeout -k 10 400 python -u tools/ab_host.py nstack_amd/libnstack_fcs.so tools/variants/libfcs_host1.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
