#!/bin/bash
# r04n: the shared-encoder split (maps and transposed convolutions in small kernels, the four products on the fp32 MFMA GEMM) of the fused ConvE path (kelpie-row, pair and relation
# terms of the FC; kp_cv_fused.hpp): the ConvE GPU parity tests, then ConvE bench lines
# with it off (KP_CV_SHARED=0) and on, alternating.
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "conve" --timeout 120 --timeout-method thread > $O/tests_conve.txt 2>&1
rc=$?
echo "conve tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $O/tests_conve.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    KP_CV_SHARED=$v timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_shared${v}_$i.json 2> $O/bench_conve_shared${v}_$i.err || exit 1
    echo "shared=$v $i $(grep -o '"value": [0-9.]*' $O/bench_conve_shared${v}_$i.json) $(grep -o '"rank_delta_match_rate[a-z_0-9]*": [0-9.]*' $O/bench_conve_shared${v}_$i.json | tr '\n' ' ')"
  done
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 6 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_conve/run_results.db --out $R/$O/conve > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_conve/run_results.db --kernel "kp_attn3<13" --window 0.4 --skip-end 0.05 \
  > $R/$O/timeline_conve.txt 2>&1 || exit 1
rm -rf $R/$O/prof_conve
head -20 $R/$O/timeline_conve.txt
# the headline: batches in flight started apart (KELPIE_PIPELINE_STAGGER_MS) or the first
# context's stream at the device's greatest priority (KP_CTX_PRIO), against neither
cd $R
for i in 1 2; do
  for v in base stagger prio; do
    case $v in base) E="" ;; stagger) E="KELPIE_PIPELINE_STAGGER_MS=7" ;; prio) E="KP_CTX_PRIO=1" ;; esac
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.json)"
  done
done
echo done
