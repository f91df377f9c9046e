set -o pipefail
bash tools/lease.sh r05p \
  "sh:tools/ab_multi.sh:r05p_ab1 c1 1 'prod||' 'p128t40|W2V_PRIV_TAIL_AVG=40|--private-rows 128'" \
  "sh:tools/ab_multi.sh:r05p_ab3 c3 1 'prod||' 'p128t40|W2V_PRIV_TAIL_AVG=40|--private-rows 128'" \
  "py:tests/probes/policy_probe.py:c1 p128t24:priv=128,W2V_PRIV_TAIL_AVG=24 p128t40:priv=128,W2V_PRIV_TAIL_AVG=40 p128t48:priv=128,W2V_PRIV_TAIL_AVG=48" \
  "py:tests/probes/policy_probe.py:c3 p128t40:priv=128,W2V_PRIV_TAIL_AVG=40" \
  "sh:tools/env_run.sh:W2V_PRIV_TAIL_AVG=24 python3 -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 private_rows=128" \
  "sh:tools/env_run.sh:W2V_PRIV_TAIL_AVG=40 python3 -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 private_rows=128" \
  "sh:tools/env_run.sh:W2V_PRIV_TAIL_AVG=48 python3 -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 private_rows=128"
