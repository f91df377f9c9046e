set -o pipefail
bash tools/lease.sh r05ay \
  "py:tests/probes/quality_paired_probe.py:text8_like cbow_hs 1,2,3 0 -;-;private_rows=64" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=4 python3 -u tests/probes/quality_paired_probe.py text8_like cbow_hs 1,2,3 0 '-;-'" \
  "sh:tools/env_run.sh:W2V_PRIV_HS_TAIL_AVG=2 python3 -u tests/probes/quality_paired_probe.py text8_like cbow_hs 1,2,3 0 '-;-'" \
  "py:tests/probes/policy_probe.py:c2 t4:W2V_PRIV_HS_TAIL_AVG=4 t2:W2V_PRIV_HS_TAIL_AVG=2"
