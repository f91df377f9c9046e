# Phase timing of the shared-negatives kernel: build a diagnostic library
# (make -C word2vec_amd/csrc prof: -DW2V_SN_PROF=1, printf of per-phase
# s_memtime sums of two workgroups) and run the configs[4] bench on it.
# usage (on the GPU box): bash tools/sn_prof.sh [bench args]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
W2V_DEV_LIB=$R/word2vec_amd/lib/prof/libw2v_hip.so timeout -k 10 200 python -u -c "
import ctypes, runpy, sys
sys.argv = ['bench.py', '--mode', 'sg_sn', '--dim', '512', '--negative', '15', '--cpu-seconds', '0', '--steps', '1', '--warmup', '0'] + sys.argv[1:]
try:
    runpy.run_path('bench.py', run_name='__main__')
finally:
    ctypes.CDLL(None).fflush(None)
" "$@" > "$R/gpurun_out/sn_prof.out" 2> "$R/gpurun_out/sn_prof.err"
grep -h SNPROF "$R/gpurun_out/sn_prof.out" "$R/gpurun_out/sn_prof.err" | head -20 || true
grep -h '"metric"' "$R/gpurun_out/sn_prof.out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'])"
