# Round 3, lease q: configs[4] quality at d512 / neg 15 — the LDS-private C rows
# (count, averaging) and more atomic rows.
set -o pipefail
TAG=${1:-r03q}
mkdir -p gpurun_out/$TAG
P="timeout -k 10 300 python -u tools/r03/c5_hot_probe.py"
$P -2 11,12 0 0 0 8 > gpurun_out/$TAG/c5_priv0.log 2>&1 || exit 1; cat gpurun_out/$TAG/c5_priv0.log
$P -2 11,12 0 0 -1 0,2,32 > gpurun_out/$TAG/c5_pavg.log 2>&1 || exit 1; cat gpurun_out/$TAG/c5_pavg.log
$P 4096,16384 11,12 0 0 -1 8 > gpurun_out/$TAG/c5_hot.log 2>&1 || exit 1; cat gpurun_out/$TAG/c5_hot.log
echo PHASE_DONE
