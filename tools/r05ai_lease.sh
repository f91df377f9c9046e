set -o pipefail
bash tools/lease.sh r05ai \
  "sh:tools/ab_multi.sh:r05ai_ab c2 2 'prod||' 'noctxat|W2V_DEV_LIB=word2vec_amd/lib/skip4/libw2v_hip.so|' 'nonodeat|W2V_DEV_LIB=word2vec_amd/lib/skip1/libw2v_hip.so|'" \
  "sh:tools/ab_multi.sh:r05ai_ab2 c2 1 'ns||--mode cbow_ns --negative 5' 'nsnoctxat|W2V_DEV_LIB=word2vec_amd/lib/skip4/libw2v_hip.so|--mode cbow_ns --negative 5'"
