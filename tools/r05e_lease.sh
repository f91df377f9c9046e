set -o pipefail
L=word2vec_amd/lib/lock/libw2v_hip.so
R=word2vec_amd/lib/rmw/libw2v_hip.so
bash tools/lease.sh r05e \
  "tests:huge_window or window_limit or outlives" \
  "sh:tools/ab_multi.sh:r05e_ab2 c2 2 'prod||' 'rmw|W2V_DEV_LIB=$R|' 'lock|W2V_DEV_LIB=$L|'" \
  "sh:tools/ab_multi.sh:r05e_ab1 c1 1 'prod||' 'lock|W2V_DEV_LIB=$L|'" \
  "sh:tools/ab_multi.sh:r05e_ab3 c3 1 'prod||' 'lock|W2V_DEV_LIB=$L|'" \
  "sh:tools/env_run.sh:W2V_DEV_LIB=$L python -u -m pytest tests/test_gpu_quality.py -m gpu -v -s --timeout 600 -k 'headline_scale or full_concurrency'"
