#!/bin/bash
# Profile the bench workload on the GPU box: kernel-trace stats, then one
# separate PMC pass per HBM counter (FETCH_SIZE and WRITE_SIZE do not fit one
# pass on gfx950; never combined with other trace domains).
# usage: tools/profile.sh <tag> [bench args...]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=("$R/bench.py" --cpu-seconds 0 "$@")
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 "${BENCH[@]}" > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python3 "${BENCH[@]}" > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python3 "${BENCH[@]}" > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
echo "profile $TAG done"
