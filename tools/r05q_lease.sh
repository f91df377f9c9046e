set -o pipefail
bash tools/lease.sh r05q "tests:headline_scale or configs3_shape or huge_window" "profile:c3" "bench:c3"
