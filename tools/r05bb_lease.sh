set -o pipefail
LEASE_PY_TIMEOUT=900 bash tools/lease.sh r05bb \
  "py:tests/probes/policy_probe.py:c3hs f256:flush=256,avg=8 f64:flush=64,avg=8 a2:avg=2 a1:avg=1 f256a2:flush=256,avg=2 f64a2:flush=64,avg=2"
