set -o pipefail
bash tools/lease.sh r05c \
  "sh:tools/ab_multi.sh:r05c_ab2 c2 2 'prod||' 'skip128|W2V_DEV_LIB=word2vec_amd/lib/skip128/libw2v_hip.so|' 'skip384|W2V_DEV_LIB=word2vec_amd/lib/skip384/libw2v_hip.so|' 'hsf32|W2V_DEV_LIB=word2vec_amd/lib/hsf32/libw2v_hip.so|'" \
  "sh:tools/ab_multi.sh:r05c_ab3 c3 2 'prod||' 'skip7|W2V_DEV_LIB=word2vec_amd/lib/skip7/libw2v_hip.so|'" \
  "sh:tools/pp_prof.sh:r05c_c2 --config c2" \
  "sh:tools/pp_prof.sh:r05c_c3 --config c3"
