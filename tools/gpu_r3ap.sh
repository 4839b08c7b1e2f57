#!/bin/bash
# Zero-copy probe: kernels reading pinned host memory over PCIe against the H2D copy engine.
set -o pipefail
out=gpurun_out/r3ap; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/zc_probe.py --gib 4 > $out/zc.log 2>&1; rc=$?
tail -5 $out/zc.log; exit $rc
