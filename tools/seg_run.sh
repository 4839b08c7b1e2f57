# GPU session for the segment kernels: parity of a variant through the dmaseg test file and the
# jumbo parity tests, then in-process A/B over lengths (measurement tool).
set -e
mkdir -p gpurun_out
V=${V:-segil}
export NSTACK_FCS_LIB=${LIB:-}
timeout -k 10 400 python -u -m pytest tests/test_gpu_segil.py tests/test_gpu_parity.py tests/test_gpu_verify.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$V.log 2>&1
for L in ${LENS:-3000 9000 10000 16500 65536}; do
  n=$(( (24 << 30) / L ))
  timeout -k 10 200 python tools/ab.py --len $L --frames $n $(for x in ${LIBS:-gen place segil}; do echo tools/variants/libfcs_$x.so; done) >> gpurun_out/ab_$V.log 2>&1
done
