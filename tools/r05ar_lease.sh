set -o pipefail
bash tools/lease.sh r05ar \
  "sh:tools/ab_multi.sh:r05ar_ab c1 1 'hs||--mode sg_hs --negative 0' 'hs96||--mode sg_hs --negative 0 --private-rows 96' 'hs128||--mode sg_hs --negative 0 --private-rows 128'" \
  "sh:tools/ab_multi.sh:r05ar_ab3 c3 1 'hs||--mode sg_hs --negative 0' 'hs127||--mode sg_hs --negative 0 --private-rows 127'"
