# CBOW-HS (c2) speed vs flush intervals of the private Huffman nodes and context rows.
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --config c2 --cpu-seconds 0 --steps 3 "$@" > gpurun_out/h2_$n.json 2> gpurun_out/h2_$n.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "$n: rc $rc $(tail -1 gpurun_out/h2_$n.err)"; [ $rc -eq 1 ] && return; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/h2_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms')"
}
run default
run sflush128 --flush-centers 128
run sflush256 --flush-centers 256
