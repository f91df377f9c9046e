#!/bin/bash
# Round-2 GPU call: the GPU test suite (no -x: every failure is reported),
# smoke(), the paired-quality probe on the text8-like corpus, the headline
# bench line, and rocprofv3 kernel-trace + FETCH/WRITE passes of the same
# workload in the same lease. usage (GPU box): bash tools/gpu_r02.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r02}
KEXPR=${2:-}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
if [ -n "$KEXPR" ]; then K=(-k "$KEXPR"); else K=(); fi
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s "${K[@]}" \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/${TAG}_gpu_tests.log | tail -2
# pytest: 0 ok, 1 failures (continue), anything else (timeout, crash) stops the call
[ $rc -le 1 ] || stop tests $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || stop smoke $?
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench $?
cat gpurun_out/${TAG}_bench_c3.json
bash tools/profile.sh ${TAG}_c3 --config c3 --steps 3 || stop profile $?
echo ALL_DONE
