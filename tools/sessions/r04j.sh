#!/bin/bash
# r04j: where the headline step's device time goes in the steady state (kernel trace of a
# 30-step run, idle-gap histogram over its middle), the same for ConvE YAGO3-10, and the
# pipeline depth (batches in flight) 3 against 4 on the headline, alternating.
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
R=$(pwd)
for i in 1 2; do
  for d in 3 4; do
    KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_depth${d}_$i.json 2> $O/bench_depth${d}_$i.err || exit 1
    echo "depth $d $i $(grep -o '"value": [0-9.]*' $O/bench_depth${d}_$i.json)"
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_default/run_results.db --out $R/$O/default > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_default/run_results.db --window 0.4 --skip-end 0.05 > $R/$O/timeline_default.txt 2>&1 || exit 1
rm -rf $R/$O/prof_default
cat $R/$O/timeline_default.txt | head -12
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 6 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_conve/run_results.db --out $R/$O/conve > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_conve/run_results.db --kernel "kp_attn3<13" --window 0.4 --skip-end 0.05 \
  > $R/$O/timeline_conve.txt 2>&1 || exit 1
rm -rf $R/$O/prof_conve
cat $R/$O/timeline_conve.txt | head -16
echo done
