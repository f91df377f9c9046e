set -o pipefail
V="p4a4:priv=4,avg=4 p4a8:priv=4,avg=8 p6a4:priv=6,avg=4 p2a4:priv=2,avg=4"
bash tools/lease.sh r05aa \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "sh:tools/ab_multi.sh:r05aa_ab c5 2 'prod||' 'p2||--private-rows 2 --private-average 4' 'p4||--private-rows 4 --private-average 4' 'p6||--private-rows 6 --private-average 4'"
