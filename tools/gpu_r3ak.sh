#!/bin/bash
# Final round-3 profile bundle on the current tree (tools/profile_round.sh).
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/prof_final > gpurun_out/prof_final.log 2>&1; rc=$?
cat gpurun_out/prof_final.log; exit $rc
