set -o pipefail
bash tools/lease.sh r05k tests "bench:c2" "sh:tools/rehearse_multi.sh:2"
