set -o pipefail
bash tools/lease.sh r05ao smoke tests "profile:c2" "bench:c2" "bench:c3"
