set -o pipefail
bash tools/lease.sh r05bg smoke "tests:headline_scale or huge_window"
