set -o pipefail
V="a1:avg=1 a2:avg=2 a4:avg=4 p128a1:priv=128,avg=1 p128a2:priv=128,avg=2 p128a4:priv=128,avg=4 w1024:waves=1024 w4096:waves=4096 w512a2:waves=512,avg=2"
bash tools/lease.sh r05au \
  "py:tests/probes/policy_probe.py:c1hs $V" \
  "py:tests/probes/policy_probe.py:c1hs $V" \
  "sh:tools/ab_multi.sh:r05au_ab c1 1 'hs||--mode sg_hs --negative 0' 'hsw512||--mode sg_hs --negative 0 --max-waves 512' 'hsw1024||--mode sg_hs --negative 0 --max-waves 1024' 'hs128||--mode sg_hs --negative 0 --private-rows 128'"
