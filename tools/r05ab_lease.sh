set -o pipefail
bash tools/lease.sh r05ab "tests:shared_negatives or sn_ or shared" "profile:c5" "bench:c5"
