set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 3 tools/variants/libfcs_nostream.so tools/variants/libfcs_stream.so tools/variants/libfcs_stnocrc.so > gpurun_out/r3c/ab.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/r3c/ab.log
bash tools/pmc.sh gpurun_out/r3c/pmc --imix --frames 33554432
python tools/pmc_summary.py gpurun_out/r3c/pmc fcs_stream_kernel > gpurun_out/r3c/pmc_stream.json; cat gpurun_out/r3c/pmc_stream.json
