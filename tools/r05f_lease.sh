set -o pipefail
LEASE_PY_TIMEOUT=1000 bash tools/lease.sh r05f \
  "sh:tools/pp_prof.sh:r05f_c2 --config c2" \
  "py:tests/probes/c3_replica_gate_probe.py:--tokens 2.5e9 --planted 0.05 --planted-sents 0.08 --ones 2 --eights 1"
