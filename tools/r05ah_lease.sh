set -o pipefail
bash tools/lease.sh r05ah "tests:huge_window"
