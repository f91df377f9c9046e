set -o pipefail
bash tools/lease.sh r05ak smoke tests "bench:c3" "bench:c5" "sh:tools/rehearse_multi.sh:2"
