# configs[1] CBOW-HS at dimensions around 200: is the kernel bound by memory
# instructions per row (64-lane dword rows: ceil(d/64) per row) or by bytes?
set -o pipefail
mkdir -p gpurun_out/dimp
for d in 128 192 200 256 320; do
  timeout -k 10 120 python bench.py --mode cbow_hs --negative 0 --vocab 250000 --tokens 17000000 --dim $d --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/dimp/d$d.json 2> gpurun_out/dimp/d$d.err || exit 1
  echo "d$d $(python -c "import json;d=json.load(open('gpurun_out/dimp/d$d.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['roofline']['avg_launch_ms'])")"
done
for d in 64 100 128; do
  timeout -k 10 120 python bench.py --mode sg_ns --negative 5 --vocab 250000 --tokens 17000000 --dim $d --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/dimp/c1d$d.json 2> gpurun_out/dimp/c1d$d.err || exit 1
  echo "c1 d$d $(python -c "import json;d=json.load(open('gpurun_out/dimp/c1d$d.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['roofline']['avg_launch_ms'])")"
done
