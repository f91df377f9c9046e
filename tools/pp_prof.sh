# Phase timing of the per-pair epoch kernel: the diagnostic library
# (make -C word2vec_amd/csrc prof: -DW2V_PP_PROF=1 for row widths 4 and 5,
# printf of per-phase s_memtime sums of some waves of two workgroups) under a
# bench run. Phases: 0 sentence loop / subsampling, 1 CBOW window set,
# 2 context gather, 3 output layer (HS / NS), 4 input-row update, 5 output-row
# flush, 6 context-row flush, 7 center bookkeeping.
# usage (on the GPU box): bash tools/pp_prof.sh <tag> [bench args]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
mkdir -p "$R/gpurun_out"
cd "$R"
W2V_DEV_LIB=${PPLIB:-$R/word2vec_amd/lib/prof/libw2v_hip.so} timeout -k 10 200 python -u -c "
import ctypes, runpy, sys
sys.argv = ['bench.py', '--cpu-seconds', '0', '--steps', '1', '--warmup', '0'] + sys.argv[1:]
try:
    runpy.run_path('bench.py', run_name='__main__')
finally:
    ctypes.CDLL(None).fflush(None)
" "$@" > "$R/gpurun_out/pp_prof_$TAG.out" 2> "$R/gpurun_out/pp_prof_$TAG.err"
grep -h PPPROF "$R/gpurun_out/pp_prof_$TAG.out" "$R/gpurun_out/pp_prof_$TAG.err" | head -40 || true
