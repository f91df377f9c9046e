# configs[1] CBOW-HS at 8 waves/SIMD (NV=4 built with W2V_MIN_WAVES=8, MAXT 2 or 4)
# with 32 + 32 private rows (64 KB: two 16-wave workgroups per CU), speed and quality.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/occ8
for v in "base:.:-1:-1" "base3232:.:32:32" "mt2:occ8mt2:32:32" "mt4:occ8mt4:32:32" "mt2_4816:occ8mt2:48:16"; do
  IFS=: read tag lib P Q <<< "$v"
  W2V_DEV_LIB=$R/word2vec_amd/lib/$lib/libw2v_hip.so timeout -k 10 120 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows $P --context-rows $Q > gpurun_out/occ8/$tag.json 2> gpurun_out/occ8/$tag.err || { echo "$tag failed"; continue; }
  echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/occ8/$tag.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['config']['policy_used'])")"
done
W2V_DEV_LIB=$R/word2vec_amd/lib/occ8mt2/libw2v_hip.so timeout -k 10 300 python -u tests/probes/quality_paired_probe.py planted cbow_hs 1,2,3 0 "private_rows=32,context_rows=32" || exit 1
W2V_DEV_LIB=$R/word2vec_amd/lib/occ8mt2/libw2v_hip.so timeout -k 10 300 python -u tests/probes/quality_paired_probe.py text8_like cbow_hs 1,2,3 0 "private_rows=32,context_rows=32" || exit 1
