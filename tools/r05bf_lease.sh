set -o pipefail
LEASE_PY_TIMEOUT=900 bash tools/lease.sh r05bf \
  "py:tests/probes/policy_probe.py:c3cbhs f256:flush=256,ctxflush=128 f64:flush=64,ctxflush=32 a4:avg=4 f256a4:flush=256,ctxflush=128,avg=4 a16:avg=16"
