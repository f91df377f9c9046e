set -o pipefail
mkdir -p gpurun_out/r03dbg
timeout -k 10 120 python -u tools/r03/pair_debug.py gpurun_out/r03dbg/pair.npz > gpurun_out/r03dbg/pair.log 2>&1 || exit 1
W2V_DEV_LIB=$PWD/word2vec_amd/lib/nopair/libw2v_hip.so timeout -k 10 120 python -u tools/r03/pair_debug.py gpurun_out/r03dbg/nopair.npz > gpurun_out/r03dbg/nopair.log 2>&1 || exit 1
echo done
