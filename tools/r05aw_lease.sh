set -o pipefail
bash tools/lease.sh r05aw smoke tests "sh:tools/ab_multi.sh:r05aw_ab c1 1 'hs||--mode sg_hs --negative 0'" "sh:tools/ab_multi.sh:r05aw_ab3 c3 1 'hs||--mode sg_hs --negative 0'" "bench:c3"
