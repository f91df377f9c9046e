set -o pipefail
LEASE_PY_TIMEOUT=900 bash tools/lease.sh r05ba \
  "py:tests/probes/policy_probe.py:c3hs prod r04:priv=64,avg=8"
