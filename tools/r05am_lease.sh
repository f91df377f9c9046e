set -o pipefail
Q="private_rows=96,context_rows=63"
bash tools/lease.sh r05am \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=40 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=128 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=0 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "py:tests/probes/policy_probe.py:c2 t40:priv=96,ctx=63,W2V_PRIV_HS_TAIL_AVG=40 t128:priv=96,ctx=63,W2V_PRIV_HS_TAIL_AVG=128" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=40 python3 -u tests/probes/quality_paired_probe.py text8_like cbow_hs 1,2,3 0 $Q" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=128 python3 -u tests/probes/quality_paired_probe.py text8_like cbow_hs 1,2,3 0 $Q"
