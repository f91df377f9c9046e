set -o pipefail
P="planted cbow_ns 1,2,3 0"
bash tools/lease.sh r05u \
  "sh:tools/env_run.sh:W2V_CTX_AVG=32 python3 -u tests/probes/quality_paired_probe.py $P 'context_rows=64,context_flush=256;context_rows=64,context_flush=64'" \
  "sh:tools/env_run.sh:W2V_CTX_AVG=128 python3 -u tests/probes/quality_paired_probe.py $P 'context_rows=64,context_flush=256;context_rows=64,context_flush=64'" \
  "sh:tools/env_run.sh:W2V_CTX_AVG=0 python3 -u tests/probes/quality_paired_probe.py $P 'context_rows=64,context_flush=256;context_rows=64,context_flush=64'" \
  "py:tests/probes/quality_paired_probe.py:$P context_rows=64,context_flush=256,private_rows=0;context_rows=16,context_flush=256;context_rows=8,context_flush=256"
