#!/bin/bash
# One runner for the GPU box (replaces the round-3 one-off session scripts):
#   bash tools/gpu_run.sh OUT STEP [STEP ...]
# Output goes under gpurun_out/OUT. Each step runs under its own time limit; the first failing
# step ends the call (no GPU step runs after a failure, a fault or a time limit). Steps:
#   suite                 the whole GPU suite (pytest -m gpu) and the graft smoke
#   tests:PATH[,PATH]     the named test files only
#   bench[:ARGS]          python bench.py ARGS (default: the driver's plain line) -> OUT/bench.json
#   ranks2                the 2-rank bench rehearsal on one GPU (bench.py --gpus 2, self-launched)
#   profile[:TAG]         tools/profile_round.sh OUT/prof TAG (trace, PMC traffic, the bundle under
#                         OUT/prof/bundle, then the plain line quoting it, rehearsals)
#   ab:ARGS               python tools/ab.py ARGS (variants built by tools/variants.sh)
#   pmc:ARGS              tools/pmc.sh OUT/pmc ARGS (SQ counter passes over tools/prof_fixed.py ARGS)
#   py:SCRIPT[,ARGS]      python SCRIPT ARGS (a measurement tool under tools/)
#   sh:CMD[,ARGS]         a tool command line (commas become spaces), e.g. sh:tools/tx_crossover,300
set -o pipefail
out=gpurun_out/${1:?usage: gpu_run.sh OUT STEP...}; shift
mkdir -p "$out"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  log="$out/$n-$kind.log"
  case $kind in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1; rc=$?
      echo "suite rc=$rc"; tail -4 "$log"; [ $rc -ne 0 ] && exit $rc
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/$n-smoke.log" 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -2 "$out/$n-smoke.log" ;;
    tests)
      timeout -k 10 900 python -u -m pytest ${arg//,/ } -x -v --timeout 300 --timeout-method thread > "$log" 2>&1; rc=$?
      echo "tests rc=$rc"; grep -E "passed|failed|error" "$log" | tail -3 ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//,/ } > "$out/$n-bench.json" 2> "$log"; rc=$?
      echo "bench rc=$rc"; tail -c 1500 "$out/$n-bench.json" ;;
    ranks2)
      timeout -k 10 600 python -u bench.py --gpus 2 --frames-per-gpu 16777216 --imix-frames-per-gpu 33554432 \
        > "$out/$n-ranks2.json" 2> "$log"; rc=$?
      echo "ranks2 rc=$rc"; tail -c 1500 "$out/$n-ranks2.json" ;;
    profile)
      timeout -k 10 1100 bash tools/profile_round.sh "$out/prof" ${arg:-r06_final} > "$log" 2>&1; rc=$?
      echo "profile rc=$rc"; tail -8 "$log" ;;
    ab)
      timeout -k 10 600 python -u tools/ab.py ${arg//,/ } > "$log" 2>&1; rc=$?
      echo "ab rc=$rc"; grep -E "GB/s|TB/s|ms" "$log" | tail -20 ;;
    pmc)
      timeout -k 10 900 bash tools/pmc.sh "$out/pmc" ${arg//,/ } > "$log" 2>&1; rc=$?
      echo "pmc rc=$rc"; tail -8 "$log" ;;
    py)
      timeout -k 10 600 python -u ${arg//,/ } > "$log" 2>&1; rc=$?
      echo "py rc=$rc"; tail -20 "$log" ;;
    sh)
      timeout -k 10 600 ${arg//,/ } > "$log" 2>&1; rc=$?
      echo "sh rc=$rc"; tail -20 "$log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  [ $rc -ne 0 ] && exit $rc
done
exit 0
