set -o pipefail
bash tools/lease.sh r05ac \
  "sh:tools/ab_multi.sh:r05ac_ab c1 1 'prod||' 'tau2||--hot-auto 2 1' 'tau4||--hot-auto 4 1' 'tau8||--hot-auto 8 1'" \
  "py:tests/probes/policy_probe.py:c1 tau2:tau=2 tau4:tau=4 tau8:tau=8" \
  "py:tests/probes/quality_paired_probe.py:text8_like sg_ns 1,2,3 0 hot_tau_rows=2;hot_tau_rows=4;hot_tau_rows=8"
