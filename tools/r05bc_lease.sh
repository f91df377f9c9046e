set -o pipefail
bash tools/lease.sh r05bc \
  "py:tests/probes/policy_probe.py:c1hs f64a2:flush=64,avg=2 f256a2:flush=256,avg=2 f64a4:flush=64,avg=4" \
  "sh:tools/ab_multi.sh:r05bc_ab3 c3 1 'hs||--mode sg_hs --negative 0' 'hsf64a2||--mode sg_hs --negative 0 --flush-centers 64 --private-average 2' 'hsf256a2||--mode sg_hs --negative 0 --flush-centers 256 --private-average 2'" \
  "py:tests/probes/quality_paired_probe.py:planted sg_hs 1,2,3 0 flush_centers=64,private_average=2"
