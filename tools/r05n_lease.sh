set -o pipefail
bash tools/lease.sh r05n "tests:quality or replica or class" "bench:c2" "profile:c2"
