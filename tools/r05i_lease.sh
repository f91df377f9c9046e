set -o pipefail
bash tools/lease.sh r05i \
  "sh:tools/ab_multi.sh:r05i_ab2 c2 1 'prod||' 'p96||--private-rows 96' 'p128||--private-rows 128' 'p96c32||--private-rows 96 --context-rows 32' 'f512||--flush-centers 512 --context-flush 256' 'prod2||'" \
  "py:tests/probes/policy_probe.py:c2 default p96:priv=96 p128:priv=128" \
  "py:tests/probes/quality_paired_probe.py:planted cbow_hs 1,2,3 0 -;private_rows=96;private_rows=128" \
  "py:tests/probes/quality_paired_probe.py:text8_like cbow_hs 1,2,3 0 -;private_rows=96;private_rows=128"
