set -o pipefail
Q="private_rows=96,context_rows=63"
bash tools/lease.sh r05an \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=4 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=2 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=1 python3 -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 $Q" \
  "py:tests/probes/policy_probe.py:c2 t4:priv=96,ctx=63,W2V_PRIV_HS_TAIL_AVG=4 t2:priv=96,ctx=63,W2V_PRIV_HS_TAIL_AVG=2 t1:priv=96,ctx=63,W2V_PRIV_HS_TAIL_AVG=1"
