set -o pipefail
bash tools/lease.sh r05t \
  "sh:tools/ab_multi.sh:r05t_ab c3 1 'prod||--mode cbow_ns' 'ctx64f256||--mode cbow_ns --context-rows 64 --context-flush 256' 'ctx64f64||--mode cbow_ns --context-rows 64 --context-flush 64' 'ctx64f32||--mode cbow_ns --context-rows 64 --context-flush 32'" \
  "py:tests/probes/quality_paired_probe.py:planted cbow_ns 1,2,3 0 -;context_rows=64,context_flush=256;context_rows=64,context_flush=64;context_rows=64,context_flush=32;context_rows=64,context_flush=16"
