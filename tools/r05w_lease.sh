set -o pipefail
V="sum256 sum64:ctxflush=64 sum128:ctxflush=128 avg128:W2V_CTX_AVG=128 avg64:W2V_CTX_AVG=64 noctx:ctx=0"
bash tools/lease.sh r05w \
  "py:tests/probes/policy_probe.py:c2ns $V" \
  "py:tests/probes/policy_probe.py:c2ns $V" \
  "py:tests/probes/policy_probe.py:c2ns $V" \
  "sh:tools/env_run.sh:W2V_CTX_AVG=64 python3 -u tests/probes/quality_paired_probe.py planted cbow_ns 1,2,3 0 'context_rows=64,context_flush=256'" \
  "py:tests/probes/quality_paired_probe.py:planted cbow_ns 1,2,3 0 context_rows=64,context_flush=128;context_rows=64,context_flush=64"
