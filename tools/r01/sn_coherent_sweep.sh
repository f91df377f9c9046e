# configs[4] bench speed vs the count of device-coherent rows (W2V_SN_COHERENT_ROWS).
set -o pipefail
mkdir -p gpurun_out
for n in 0 16 64 256 1024 4096; do
W2V_SN_COHERENT_ROWS=$n timeout -k 10 200 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 0 --steps 2 > gpurun_out/bench_cr$n.json 2> gpurun_out/bench_cr$n.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_cr$n.json'));print('coherent rows $n', d['value'], d['roofline']['frac'])"
done
