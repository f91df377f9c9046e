set -o pipefail
mkdir -p gpurun_out
for o in 0 3 4; do
  W2V_SN_OCC=$o timeout -k 10 200 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 0 --steps 2 > gpurun_out/sn_occ$o.json 2> gpurun_out/sn_occ$o.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sn_occ$o.json'));print('occ $o', d['value'], d['roofline']['frac'], d['roofline']['mfma']['frac'])"
done
