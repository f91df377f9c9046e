#!/bin/bash
# One GPU lease, parameterised: the steps run in order on the GPU box, each
# under its own time limit, and the lease stops at the first failing step
# (a GPU fault, abort or time limit ends the call there).
# usage (through gpurun, from the repo root):
#   tools/lease.sh <tag> <step> [<step> ...]
# steps:
#   smoke                     __graft_entry__.smoke()
#   tests[:<pytest -k expr>]  the GPU suite (or the selected tests), no -x, every failure reported
#   bench:<cN>[:<args>]       one bench.py line of a BASELINE preset (extra args space-separated)
#   profile:<cN>              tools/profile.sh (kernel trace + FETCH_SIZE + WRITE_SIZE passes) +
#                             tools/pmc_summary.py -> profiles/<tag>_<cN>_* and profiles/pmc_traffic.json
#   pmc:<cN>[:<passes>]       tools/pmc.sh counter passes (default sq1 sq2 tcc atom)
#   py:<script>[:<args>]      python3 -u <script> <args> (600 s; LEASE_PY_TIMEOUT overrides) -> <tag>_<step#>_<script>.log
#   sh:<script>[:<args>]      bash <script> <args> (900 s), e.g. sh:tools/r03/ab.sh:<tag> <variant> "c3 c1" 2
# Outputs: gpurun_out/<tag>_*; profiles written on the box come back under
# gpurun_out/<tag>_profiles/ (copy them into profiles/ to commit).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT/${TAG}_profiles
stop() { echo "STOP at step '$1' (rc=$2)"; exit 1; }
n=0
for step in "$@"; do
  n=$((n + 1))
  IFS=: read -r kind a b <<< "$step"
  echo "== $step ($(date +%T))"
  case $kind in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || stop "$step" $?
      tail -1 $OUT/${TAG}_smoke.log ;;
    tests)
      sel=(); [ -n "$a" ] && sel=(-k "$a")
      W2V_PARITY_LOG=$PWD/$OUT/${TAG}_parity_errors.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s \
        --timeout 300 --timeout-method thread "${sel[@]}" > $OUT/${TAG}_tests.log 2>&1
      rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/${TAG}_tests.log | tail -12
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || stop "$step" $rc ;;
    bench)
      timeout -k 10 500 python -u bench.py --config $a $b > $OUT/${TAG}_bench_$a.json 2> $OUT/${TAG}_bench_$a.err || stop "$step" $?
      cat $OUT/${TAG}_bench_$a.json ;;
    profile)
      bash tools/profile.sh ${TAG}_$a --config $a --steps 3 || stop "$step" $?
      python tools/pmc_summary.py ${TAG}_$a > $OUT/${TAG}_pmc_summary_$a.log 2>&1 || stop "$step" $?
      cp profiles/${TAG}_${a}_kernel_stats.csv profiles/${TAG}_${a}_pmc.json profiles/pmc_traffic.json $OUT/${TAG}_profiles/
      grep -E "avg_duration_ms_rocprof|hbm_traffic_bytes_per_launch\"|algorithmic" $OUT/${TAG}_pmc_summary_$a.log ;;
    pmc)
      PASSES="${b:-sq1 sq2 tcc atom}" bash tools/pmc.sh ${TAG}_$a --config $a || stop "$step" $?
      python tools/pmc_table.py ${TAG}_$a > $OUT/${TAG}_pmc_table_$a.log 2>&1 || true
      cat $OUT/${TAG}_pmc_table_$a.log ;;
    py)
      log=$OUT/${TAG}_${n}_$(basename $a .py).log
      timeout -k 10 ${LEASE_PY_TIMEOUT:-600} python3 -u $a $b > $log 2>&1 || stop "$step" $?
      tail -12 $log ;;
    sh)
      log=$OUT/${TAG}_${n}_$(basename $a .sh).log
      eval "timeout -k 10 900 bash $a $b" > $log 2>&1 || stop "$step" $?
      tail -20 $log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo LEASE_DONE
