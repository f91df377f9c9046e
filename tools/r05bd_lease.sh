set -o pipefail
LEASE_PY_TIMEOUT=900 bash tools/lease.sh r05bd \
  "py:tests/probes/policy_probe.py:c3hs w4096:waves=4096 w2048:waves=2048 w1024:waves=1024" \
  "py:tests/probes/policy_probe.py:c1hs w4096:waves=4096 w2048:waves=2048"
