set -o pipefail
bash tools/lease.sh r05aq "sh:tools/rehearse_multi.sh:4"
