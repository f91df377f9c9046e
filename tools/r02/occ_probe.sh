# configs[1] CBOW-HS: waves per SIMD (register budget, W2V_MIN_WAVES builds
# under word2vec_amd/lib/occN) x LDS per workgroup (private rows) x workgroup size.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/occ
run() {  # tag lib wpb lds_per_wave
  W2V_DEV_LIB=$R/word2vec_amd/lib/$2/libw2v_hip.so W2V_DEBUG_WPB=$3 W2V_DEBUG_LDS_PER_WAVE=$4 \
    timeout -k 10 120 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/occ/$1.json 2> gpurun_out/occ/$1.err || return 1
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/occ/$1.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['config']['policy_used'])")"
}
run base_16_10k . 16 10240 && run base_16_4k . 16 4096 && run base_8_6k . 8 6144 && \
run occ6_8_6k occ6 8 6144 && run occ6_16_10k occ6 16 10240 && \
run occ8_16_4k occ8 16 4096 && run occ8_8_4k occ8 8 4096 && run occ8_16_10k occ8 16 10240
