# Headline kernel: the next item's DMA issued before the chain (product) or after 3 / 6 / 9 of its
# 12 steps (fewer bytes in flight per CU), one process.
set -o pipefail
out=gpurun_out/r3s; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab.py --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_iss3.so tools/variants/libfcs_iss6.so tools/variants/libfcs_iss9.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
