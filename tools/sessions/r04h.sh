#!/bin/bash
# r04h: where the headline's round-4 wall-clock regression comes from.  Alternating on one
# box: the round-3 library, this tree with the round-3 ComplEx kernels (kp_complex.hip of
# round 3 compiled against today's headers: variants/lib_cx03.so) and this tree; then a
# kernel trace of the round-3 library and of this tree (summaries only: the raw SQLite
# outputs are deleted on the box), and the ConvE counter passes of r04f (lost: its raw
# outputs exceeded the copy-back limit).
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
R=$(pwd)
lib() { case $1 in r03) echo $R/variants/lib_r03.so ;; cx03) echo $R/variants/lib_cx03.so ;; *) echo $R/kelpie_amd/libkelpie_hip.so ;; esac; }
for i in 1 2; do
  for v in r03 cx03 cur; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    echo "$v $i $(cut -c1-120 $O/bench_${v}_$i.json | grep -o '"value": [0-9.]*')"
  done
done
export TMPDIR=/tmp
cd /tmp
for v in r03 cur; do
  KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof_$v.log 2>&1 || exit 1
  python3 $R/tools/prof_summary.py --stats $R/$O/prof_$v/run_results.db --out $R/$O/$v > /dev/null || exit 1
  python3 $R/tools/timeline.py $R/$O/prof_$v/run_results.db > $R/$O/timeline_$v.txt 2>&1 || exit 1
  rm -rf $R/$O/prof_$v
done
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "kp_cv_|kp_attn3" -d $R/$O/pmc_conve_p$i -o run -- \
    python3 $R/bench.py --workload conve-yago310-necessary --steps 1 --warmup 1 --no-cpu-baseline > $R/$O/pmc_conve_p$i.log 2>&1 || exit 1
  python3 $R/tools/pmc_dump.py $R/$O/pmc_conve_p$i/run_results.db > $R/$O/pmc_conve_p$i.txt || exit 1
  rm -rf $R/$O/pmc_conve_p$i
  i=$((i + 1))
done
cat $R/$O/pmc_conve_p*.txt | grep -E "fwd_fused|bwd_fused" | cut -c1-140
echo done
