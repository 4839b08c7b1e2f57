# Stream kernel ablations (one A/B process) and two PMC passes of the product stream kernel on IMIX.
set -o pipefail
out=gpurun_out/r3i; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_nostream.so tools/variants/libfcs_stnocrc.so tools/variants/libfcs_stnoclose.so tools/variants/libfcs_stnoshift.so tools/variants/libfcs_stbare.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -7; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p1 -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 tools/prof_fixed.py --reps 2 --imix --frames 134217728 > $out/p1.log 2>&1; rc=$?
echo "p1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p2 -o run --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD -- python3 tools/prof_fixed.py --reps 2 --imix --frames 134217728 > $out/p2.log 2>&1; rc=$?
echo "p2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_summary.py $out fcs_stream_kernel > $out/pmc_stream.json; cat $out/pmc_stream.json
