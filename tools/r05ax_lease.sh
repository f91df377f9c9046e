set -o pipefail
bash tools/lease.sh r05ax smoke tests "bench:c3"
