set -o pipefail
bash tools/lease.sh r05as \
  "py:tests/probes/policy_probe.py:c1hs prod p96:priv=96 p128:priv=128" \
  "py:tests/probes/policy_probe.py:c1hs prod p96:priv=96 p128:priv=128" \
  "py:tests/probes/quality_paired_probe.py:planted sg_hs 1,2,3 0 -;private_rows=96;private_rows=128"
