set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dmaseg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dmaseg.log 2>&1
for L in 3000 4500 6000 9000 16500 41148; do
  n=$(( (24 << 30) / L ))
  timeout -k 10 200 python tools/ab.py --len $L --frames $n tools/variants/libfcs_{gen,carry,place}.so >> gpurun_out/ab_place.log 2>&1
done
