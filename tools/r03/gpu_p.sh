# Round 3, lease p: configs[4] quality at d512 / neg 15 vs concurrency and step size.
set -o pipefail
TAG=${1:-r03p}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u tools/r03/c5_hot_probe.py -2 11,12 0,1024,256,64,2 0 > gpurun_out/$TAG/c5_waves.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_waves.log
timeout -k 10 300 python -u tools/r03/c5_hot_probe.py -2 11,12 0 0.0125,0.05 > gpurun_out/$TAG/c5_alpha.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_alpha.log
echo PHASE_DONE
