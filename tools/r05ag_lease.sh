set -o pipefail
bash tools/lease.sh r05ag smoke tests "bench:c3"
