#!/bin/bash
# Round-2 GPU calls (each phase fits one gpurun call of <= 1200 s).
#   bash tools/gpu_r02.sh <tag> tests [pytest -k expr]   the GPU test suite (no -x: every failure reported)
#   bash tools/gpu_r02.sh <tag> bench                    smoke(), the headline bench line, then rocprofv3
#                                                        kernel-trace + FETCH/WRITE passes of the same workload
#   bash tools/gpu_r02.sh <tag> probe "<probe args>"     tests/probes/quality_paired_probe.py
set -o pipefail
TAG=${1:-r02}
PHASE=${2:-tests}
ARG=${3:-}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
case $PHASE in
tests)
  if [ -n "$ARG" ]; then K=(-k "$ARG"); else K=(); fi
  timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s "${K[@]}" \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/${TAG}_gpu_tests.log | tail -2
  grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_gpu_tests.log | head -40
  # pytest: 0 ok, 1 failures; anything else (timeout, crash) is reported as such
  [ $rc -le 1 ] || stop tests $rc
  ;;
bench)
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || stop smoke $?
  timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench $?
  cat gpurun_out/${TAG}_bench_c3.json
  bash tools/profile.sh ${TAG}_c3 --config c3 --steps 3 || stop profile $?
  ;;
probe)
  timeout -k 10 1080 python -u tests/probes/quality_paired_probe.py $ARG > gpurun_out/${TAG}_probe.log 2>&1 || stop probe $?
  cat gpurun_out/${TAG}_probe.log
  ;;
esac
echo PHASE_DONE
