#!/bin/bash
# r04f: the full-size parity table (every fixture against the reference variants), the
# counter passes of the fused ConvE encoder kernels as shipped, and the bench lines of
# the other workloads.
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u tools/fullsize_table.py > $O/fullsize_table.jsonl 2> $O/fullsize_table.err || { tail -5 $O/fullsize_table.err; exit 1; }
cut -c1-220 $O/fullsize_table.jsonl
for w in conve-yago310-necessary transe-fb15k237-necessary complex-fb15k237-necessary complex-db100k-sufficient; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  cut -c1-160 $O/bench_$w.json
done
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES"; do
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "kp_cv_|kp_attn3" -d $R/$O/pmc_conve_p$i -o run -- \
    python3 $R/bench.py --workload conve-yago310-necessary --steps 1 --warmup 1 --no-cpu-baseline > $R/$O/pmc_conve_p$i.log 2>&1 || exit 1
  i=$((i + 1))
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
echo done
