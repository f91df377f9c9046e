set -o pipefail
bash tools/lease.sh r05ap \
  "sh:tools/ab_multi.sh:r05ap_ab c2 1 'ns||--mode cbow_ns --negative 5' 'ns95||--mode cbow_ns --negative 5 --private-rows 95'" \
  "sh:tools/ab_multi.sh:r05ap_ab3 c3 1 'ns||--mode cbow_ns' 'ns96q31||--mode cbow_ns --private-rows 96 --context-rows 31'" \
  "py:tests/probes/policy_probe.py:c2ns p95:priv=95 p95b:priv=95 p95t8:priv=95,W2V_PRIV_TAIL_AVG=8"
