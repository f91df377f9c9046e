set -o pipefail
bash tools/lease.sh r05b "tests:c5_hyperparameters or outlives or shared_negatives" \
  "py:tests/probes/divergence_gpu_probe.py:priv0:priv=0 flush16:flush=16 flush4:flush=4 avg0:avg=0 w64priv0:waves=64,priv=0 w16priv0:waves=16,priv=0" \
  "py:tests/probes/policy_probe.py:c5 default default2" \
  "py:tests/probes/limits_cost_probe.py" \
  "sh:tools/ab_multi.sh:r05b_ab c2 2 'prod||' 'skip7|W2V_DEV_LIB=word2vec_amd/lib/skip7/libw2v_hip.so|' 'skip71|W2V_DEV_LIB=word2vec_amd/lib/skip71/libw2v_hip.so|'" \
  "sh:tools/ab_multi.sh:r05b_ab1 c1 2 'prod||' 'skip7|W2V_DEV_LIB=word2vec_amd/lib/skip7/libw2v_hip.so|' 'skip71|W2V_DEV_LIB=word2vec_amd/lib/skip71/libw2v_hip.so|'"
