#!/bin/bash
# PMC passes over one bench workload (each pass its own rocprofv3 run, counters
# within the per-block limits of MI355X_MICROARCH.md; never combined with trace
# domains). usage (GPU box): tools/pmc.sh <tag> [bench args...]
# -> gpurun_out/pmc_<tag>/<pass>/... ; summarise with tools/pmc_table.py <tag>
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=("$R/bench.py" --cpu-seconds 0 --steps 1 --warmup 0 "$@")
declare -A PASS
PASS[sq1]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
PASS[sq2]="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
PASS[tcc]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_avr"
PASS[fetch]="FETCH_SIZE"
PASS[write]="WRITE_SIZE"
PASS[atom]="TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"
for p in ${PASSES:-sq1 sq2 tcc fetch write}; do
  timeout -s KILL 120 rocprofv3 --pmc ${PASS[$p]} --output-format csv -d "$OUT/$p" -o $p -- python3 "${BENCH[@]}" > "$OUT/$p.json" 2> "$OUT/$p.err"
  echo "pass $p done"
done
