set -o pipefail
bash tools/lease.sh r05at \
  "py:tests/probes/policy_probe.py:c1hs prod priv0:priv=0 f64:flush=64 f1024:flush=1024 avg2:avg=2 avg32:avg=32 w2048:waves=2048 w512:waves=512 w128:waves=128 tau4:tau=1,tau_nodes=4 tau025:tau=1,tau_nodes=0.25"
