# A/B of measurement libraries on the GPU box (tools/ab.py), output under gpurun_out/$1
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 500 python tools/ab.py "$@" > $out/ab.log 2>&1; rc=$?
tail -30 $out/ab.log; exit $rc
