set -o pipefail
bash tools/lease.sh r05x smoke tests \
  "sh:tools/ab_multi.sh:r05x_ab c3 1 'cbowns||--mode cbow_ns'" \
  "sh:tools/ab_multi.sh:r05x_ab2 c2 1 'cbowns||--mode cbow_ns --negative 5'" \
  "bench:c3"
