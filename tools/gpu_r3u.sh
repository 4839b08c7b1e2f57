set -o pipefail
out=gpurun_out/r3u; mkdir -p $out
NSTACK_FCS_TRACE_HOST=1 timeout -k 10 100 python -u tools/host_chunks_probe.py shuffled 2>&1 | tee $out/probe.log; exit ${PIPESTATUS[0]}
