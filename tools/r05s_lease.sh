set -o pipefail
bash tools/lease.sh r05s smoke tests "profile:c1" "bench:c1" "bench:c3"
