set -o pipefail
bash tools/lease.sh r05aj \
  "sh:tools/ab_multi.sh:r05aj_ab c5 1 'prod||' 'at500|W2V_SN_ATOMIC_ROWS=500|' 'at2000|W2V_SN_ATOMIC_ROWS=2000|' 'p6||--private-rows 6'" \
  "py:tests/probes/policy_probe.py:c5 at500:W2V_SN_ATOMIC_ROWS=500 at2000:W2V_SN_ATOMIC_ROWS=2000"
