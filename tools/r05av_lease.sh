set -o pipefail
bash tools/lease.sh r05av \
  "py:tests/probes/quality_paired_probe.py:planted sg_hs 1,2,3 0 private_rows=128,private_average=4;private_rows=128,private_average=2;private_rows=64,private_average=4" \
  "sh:tools/ab_multi.sh:r05av_ab c3 1 'hs||--mode sg_hs --negative 0' 'hs127a4||--mode sg_hs --negative 0 --private-rows 127 --private-average 4'" \
  "py:tests/probes/policy_probe.py:c1hs p128a4:priv=128,avg=4 p128a3:priv=128,avg=3"
