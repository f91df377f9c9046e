# Round 3, lease b: the whole GPU suite (no -x: every failure listed) with the
# measured parity errors logged, the small-corpus full-concurrency regression
# probes, and the 8-replica exchange study.
set -o pipefail
TAG=${1:-r03b}
mkdir -p gpurun_out/$TAG
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
rm -f gpurun_out/$TAG/parity_errors.jsonl
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -15
[ $rc -le 1 ] || stop gpu_tests $rc
timeout -k 10 500 python -u tests/probes/quality_paired_probe.py text8_small sg_ns,cbow_hs 1 0,1024,512,256 "-;private_rate=0.1" > gpurun_out/$TAG/small.log 2>&1 || stop small $?
cat gpurun_out/$TAG/small.log
timeout -k 10 400 python -u tests/probes/quality_paired_probe.py planted sg_ns,sg_hs,cbow_ns,cbow_hs 1 0 "-;private_rate=0.1" > gpurun_out/$TAG/planted.log 2>&1 || stop planted $?
cat gpurun_out/$TAG/planted.log
timeout -k 10 900 python -u tools/r03/replica_study.py --tokens 50000000 --replicas 8 --rounds 1,8,32,128 --gmodes sum,average,row_average > gpurun_out/$TAG/replicas_sg_ns.log 2>&1 || stop replicas $?
cat gpurun_out/$TAG/replicas_sg_ns.log
