set -o pipefail
V="prod p10a8:priv=10 p10a128:priv=10,avg=128 p10a128f256:priv=10,avg=128,flush=256 p10sum:priv=10,avg=0 p4a128:priv=4,avg=128"
bash tools/lease.sh r05y \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "sh:tools/ab_multi.sh:r05y_ab c5 1 'prod||' 'p10||--private-rows 10 --private-average 128' 'p4||--private-rows 4 --private-average 128'"
