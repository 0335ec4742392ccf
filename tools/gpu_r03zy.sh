#!/bin/bash
# r03zy: counter passes of the attention micro-benchmark at the settled clock (1 s of launches
# before the timed ones), FB15k-237 shape; each pass its own run
set -o pipefail
O=gpurun_out/r03zy; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $R/$O/p$i -o run -- $R/variants/attn_micro_base 25 0 14541 3100 30 0.05 > $R/$O/p$i.log 2>&1 || exit 1
  i=$((i + 1))
done
cd $R
for i in 0 1; do python tools/pmc_dump.py $O/p$i/run_results.db kp_attn3 | tee -a $O/summary.txt; done
