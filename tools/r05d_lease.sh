set -o pipefail
R=word2vec_amd/lib/rmw/libw2v_hip.so
timeout -k 10 120 ./tools/lds_atomic_bench > gpurun_out/r05d_lds_atomic_bench.log 2>&1 && cat gpurun_out/r05d_lds_atomic_bench.log
bash tools/lease.sh r05d \
  "sh:tools/ab_multi.sh:r05d_ab2 c2 2 'prod||' 'rmw|W2V_DEV_LIB=$R|'" \
  "sh:tools/ab_multi.sh:r05d_ab1 c1 2 'prod||' 'rmw|W2V_DEV_LIB=$R|' 'skip128|W2V_DEV_LIB=word2vec_amd/lib/skip128/libw2v_hip.so|'" \
  "sh:tools/ab_multi.sh:r05d_ab3 c3 1 'prod||' 'rmw|W2V_DEV_LIB=$R|' 'skip128|W2V_DEV_LIB=word2vec_amd/lib/skip128/libw2v_hip.so|' 'hot0||--hot-rows 0' 'skip7|W2V_DEV_LIB=word2vec_amd/lib/skip7/libw2v_hip.so|'" \
  "py:tests/probes/divergence_gpu_probe.py:w1:waves=1 w2:waves=2 w4:waves=4 w8:waves=8 w1p0:waves=1,priv=0 w4p0:waves=4,priv=0" \
  "sh:tools/env_run.sh:W2V_DEV_LIB=$R python -u -m pytest tests/test_gpu_quality.py -m gpu -v -s --timeout 600 -k 'headline_scale or full_concurrency'"
