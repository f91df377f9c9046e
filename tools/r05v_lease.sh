set -o pipefail
bash tools/lease.sh r05v \
  "py:tests/probes/policy_probe.py:c2ns prod noctx:ctx=0 ctxavg8:W2V_CTX_AVG=8 ctxf64:ctxflush=64" \
  "sh:tools/ab_multi.sh:r05v_ab c3 1 'prod||--mode cbow_ns' 'noctx||--mode cbow_ns --context-rows 0'" \
  "sh:tools/ab_multi.sh:r05v_ab2 c2 1 'prod||--mode cbow_ns --negative 5' 'noctx||--mode cbow_ns --negative 5 --context-rows 0'" \
  "tests:cbow_ns or cbow-ns or c2ns or planted_not_below"
