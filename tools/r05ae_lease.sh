set -o pipefail
bash tools/lease.sh r05ae "tests:replicas or shared_negatives" "bench:c5"
