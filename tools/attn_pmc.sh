#!/bin/bash
# Counter passes over one bench workload's attention launches (GPU box), each its own run:
#   bash tools/attn_pmc.sh <out-dir> <workload> [extra env assignments for bench]
# Summaries: python tools/pmc_dump.py <out-dir>/<pass>/run_results.db kp_attn
set -eo pipefail
OUT=$1
WL=$2
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for P in "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 150 rocprofv3 --pmc $P -d "$ROOT/$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/p$i.log" 2>&1
  i=$((i + 1))
done
