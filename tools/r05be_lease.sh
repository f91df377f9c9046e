set -o pipefail
LEASE_PY_TIMEOUT=900 bash tools/lease.sh r05be \
  "py:tests/probes/policy_probe.py:c3cbhs prod ctx0:ctx=0"
