set -o pipefail
O5=word2vec_amd/lib/occ5/libw2v_hip.so
O6=word2vec_amd/lib/occ6/libw2v_hip.so
bash tools/lease.sh r05h \
  "sh:tools/ab_multi.sh:r05h_ab2 c2 1 'prod||' 'tn2||--hot-auto 0 2' 'tn4||--hot-auto 0 4' 'tn8||--hot-auto 0 8' 'tr2tn2||--hot-auto 2 2' 'tr4tn4||--hot-auto 4 4' 'hot0||--hot-rows 0' 'occ5|W2V_DEV_LIB=$O5 W2V_DEBUG_WPB=10 W2V_DEBUG_LDS_PER_WAVE=8000|' 'occ6|W2V_DEV_LIB=$O6 W2V_DEBUG_WPB=12 W2V_DEBUG_LDS_PER_WAVE=6600|' 'prod2||'"
