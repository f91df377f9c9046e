set -o pipefail
bash tools/lease.sh r05l smoke "profile:c3" "profile:c2" "bench:c3"
