set -o pipefail
bash tools/lease.sh r05ad smoke tests "profile:c3" "profile:c2" "bench:c3" "bench:c1" "bench:c2" "bench:c5" \
  "sh:tools/rehearse_multi.sh:2"
