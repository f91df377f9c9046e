set -o pipefail
bash tools/lease.sh r05af "pmc:c2:sq1 sq2 tcc atom" "pmc:c1:sq1 tcc atom" "pmc:c3:sq1 atom" "pmc:c5:sq1 atom"
