#!/bin/bash
# r04p: the transposed convolutions with their ReLU bytes staged in LDS: ConvE GPU tests,
# two ConvE bench lines and a ConvE trace; then the headline trace with its idle gaps listed.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "conve" --timeout 120 --timeout-method thread > $O/tests_conve.txt 2>&1
rc=$?
echo "conve tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $O/tests_conve.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
    --no-cpu-baseline > $O/bench_conve_$i.json 2> $O/bench_conve_$i.err || exit 1
  echo "conve $i $(grep -o '"value": [0-9.]*' $O/bench_conve_$i.json) $(grep -o '"rank_delta_match_rate_ref_fp64": [0-9.]*' $O/bench_conve_$i.json)"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 6 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_conve/run_results.db --out $R/$O/conve > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_conve/run_results.db --kernel "kp_attn3<13" --window 0.4 --skip-end 0.05 \
  > $R/$O/timeline_conve.txt 2>&1 || exit 1
rm -rf $R/$O/prof_conve
head -20 $R/$O/timeline_conve.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_default/run_results.db --out $R/$O/default > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_default/run_results.db --window 0.4 --skip-end 0.05 --gaps > $R/$O/timeline_default.txt 2>&1 || exit 1
rm -rf $R/$O/prof_default
head -24 $R/$O/timeline_default.txt
echo done
