#!/bin/bash
# r04f: the headline A/B of the round-3 library against this tree's (kp_cx_prep folded
# back into kp_cx_contrib), alternating on one box, with a kernel trace of the default
# bench; ConvE with the spread LDS-DMA under lgkmcnt(0) / vmcnt(0) against the burst;
# the counter passes of the fused ConvE encoder kernels as shipped, and the bench lines of
# the other workloads.
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
R=$(pwd)
for i in 1 2; do
  for v in r03 cur; do
    L=$R/kelpie_amd/libkelpie_hip.so; [ $v = r03 ] && L=$R/variants/lib_r03.so
    KELPIE_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    cut -c1-200 $O/bench_${v}_$i.json
  done
done
for i in 1 2; do
  for v in cur spr_lgkm0 spr_vm0; do
    L=$R/kelpie_amd/libkelpie_hip.so; [ $v != cur ] && L=$R/variants/lib_$v.so
    KELPIE_HIP_LIB=$L timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_${v}_$i.json 2> $O/bench_conve_${v}_$i.err || exit 1
    cut -c1-200 $O/bench_conve_${v}_$i.json
  done
done
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES"; do
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "kp_cv_|kp_attn3" -d $R/$O/pmc_conve_p$i -o run -- \
    python3 $R/bench.py --workload conve-yago310-necessary --steps 1 --warmup 1 --no-cpu-baseline > $R/$O/pmc_conve_p$i.log 2>&1 || exit 1
  i=$((i + 1))
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
echo done
