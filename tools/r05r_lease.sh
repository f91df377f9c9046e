set -o pipefail
bash tools/lease.sh r05r \
  "sh:tools/ab_multi.sh:r05r_ab1 c1 1 'prod||' 'p96|W2V_PRIV_TAIL_AVG=40|--private-rows 96' 'p112|W2V_PRIV_TAIL_AVG=40|--private-rows 112'" \
  "py:tests/probes/policy_probe.py:c1 p96t32:priv=96,W2V_PRIV_TAIL_AVG=32 p96t40:priv=96,W2V_PRIV_TAIL_AVG=40 p112t40:priv=112,W2V_PRIV_TAIL_AVG=40" \
  "sh:tools/env_run.sh:W2V_PRIV_TAIL_AVG=40 python3 -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 'private_rows=96;private_rows=112'" \
  "sh:tools/env_run.sh:W2V_PRIV_TAIL_AVG=32 python3 -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 private_rows=96"
