set -o pipefail
out=gpurun_out/r3v; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "host or tx" tests/test_gpu_multidev_alias.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu > $out/bench.json 2> $out/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['roofline']['frac'])
for k,v in d['configs'].items(): print(k, v.get('GB_s'), v.get('ms'), v['roofline'].get('frac_of_h2d_copy'), v['roofline'].get('h2d_copy_gbs'), v['roofline'].get('h2d_copy_s'))"
exit $rc
