# Host pipeline (per-buffer streams, fast chunking): host-path parity tests, then the bench line.
set -o pipefail
out=gpurun_out/r3t; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "host or tx" tests/test_gpu_multidev_alias.py tests/test_gpu_txq.py tests/test_gpu_rxq.py tests/test_gpu_pcap.py tests/test_gpu_inet.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['roofline']['frac'])
for k,v in d['configs'].items(): print(k, v.get('GB_s'), v['roofline'].get('frac_of_h2d_copy'), v['roofline'].get('frac_of_dma_stream'))"
exit $rc
