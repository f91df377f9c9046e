set -o pipefail
LEASE_PY_TIMEOUT=1000 bash tools/lease.sh r05g \
  "sh:tools/ab_multi.sh:r05g_ab2 c2 2 'prod||' 'skip7|W2V_DEV_LIB=word2vec_amd/lib/skip7/libw2v_hip.so|' 'skip71|W2V_DEV_LIB=word2vec_amd/lib/skip71/libw2v_hip.so|'" \
  "py:tests/probes/c3_replica_gate_probe.py:--tokens 2.5e9 --planted 0.05 --planted-sents 0.02 --ones 2 --eights 1" \
  "py:tests/probes/c3_replica_gate_probe.py:--tokens 2.5e9 --planted 0.05 --planted-sents 0.01 --ones 2 --eights 1"
