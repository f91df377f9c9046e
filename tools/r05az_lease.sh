set -o pipefail
bash tools/lease.sh r05az smoke tests "bench:c2" "bench:c3"
