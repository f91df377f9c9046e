set -o pipefail
bash tools/lease.sh r05m "profile:c1" "profile:c5" "bench:c1" "bench:c2" "bench:c5" \
  "py:tests/probes/quality_paired_probe.py:planted sg_hs,cbow_hs 1,2,3 0 -;flush_centers=128,context_flush=64" \
  "py:tests/probes/quality_paired_probe.py:text8_like cbow_hs 1,2,3 0 flush_centers=1024,context_flush=512"
