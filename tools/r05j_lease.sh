set -o pipefail
bash tools/lease.sh r05j \
  "sh:tools/ab_multi.sh:r05j_ab2 c2 1 'prod||' 'f512||--flush-centers 512 --context-flush 256' 'f1024||--flush-centers 1024 --context-flush 512' 'f512c512||--flush-centers 512 --context-flush 512'" \
  "py:tests/probes/policy_probe.py:c2 f512:flush=512,ctxflush=256 f1024:flush=1024,ctxflush=512 f512c512:flush=512,ctxflush=512" \
  "py:tests/probes/quality_paired_probe.py:text8_like cbow_hs 1,2,3 0 flush_centers=256,context_flush=128;flush_centers=512,context_flush=256" \
  "py:tests/probes/quality_paired_probe.py:text8_small cbow_hs 1 0 -;flush_centers=256,context_flush=128;flush_centers=512,context_flush=256"
