# Shared-negatives staged atomic rows: private rows combos (quality+speed), atomic-row counts (speed).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/sn_private_sweep.py 0,0 4,1024 4,256 2,1024 > gpurun_out/snp3.log 2>&1 || { cat gpurun_out/snp3.log; exit 1; }
cat gpurun_out/snp3.log
for h in 300 3000; do W2V_SN_ATOMIC_ROWS=$h timeout -k 10 200 python -u bench.py --config c5 --cpu-seconds 0 --steps 2 > gpurun_out/c5_h$h.json 2>gpurun_out/c5_h$h.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/c5_h$h.json'));print('atomic rows $h', round(d['value']/1e6,1))"; done
