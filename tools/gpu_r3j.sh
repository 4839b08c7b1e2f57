# Stream kernel with skewed hole tables: parity, A/B against the unskewed build and the flat kernel, conflicts.
set -o pipefail
out=gpurun_out/r3j; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_windowed.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_stnoskew.so tools/variants/libfcs_nostream.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p2 -o run --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD -- python3 tools/prof_fixed.py --reps 2 --imix --frames 134217728 > $out/p2.log 2>&1; rc=$?
echo "p2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_summary.py $out fcs_stream_kernel > $out/pmc_stream.json; cat $out/pmc_stream.json
