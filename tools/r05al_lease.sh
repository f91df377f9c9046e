set -o pipefail
bash tools/lease.sh r05al \
  "sh:tools/ab_multi.sh:r05al_ab c2 1 'prod||' 'p96q63||--private-rows 96 --context-rows 63' 'p96q32||--private-rows 96 --context-rows 32' 'p128q32||--private-rows 128 --context-rows 31'" \
  "py:tests/probes/policy_probe.py:c2 p96q63:priv=96,ctx=63 p96q32:priv=96,ctx=32 p128q31:priv=128,ctx=31" \
  "py:tests/probes/quality_paired_probe.py:text8_like cbow_hs 1,2,3 0 private_rows=96,context_rows=63;private_rows=96,context_rows=32;private_rows=128,context_rows=31" \
  "py:tests/probes/quality_paired_probe.py:planted cbow_hs 1,2,3 0 private_rows=96,context_rows=63;private_rows=96,context_rows=32;private_rows=128,context_rows=31"
