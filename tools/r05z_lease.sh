set -o pipefail
V="p10a4:priv=10,avg=4 p10a2:priv=10,avg=2 p10a4f256:priv=10,avg=4,flush=256 p10a8f256:priv=10,avg=8,flush=256 p4a4:priv=4,avg=4 p10a1:priv=10,avg=1"
bash tools/lease.sh r05z \
  "py:tests/probes/policy_probe.py:c5 $V" \
  "py:tests/probes/policy_probe.py:c5 $V"
