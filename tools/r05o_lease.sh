set -o pipefail
bash tools/lease.sh r05o smoke tests "bench:c3"
