#!/bin/bash
# r04z2: closing measurements of round 4 on the final library, one box: smoke(); the default bench line as the
# driver runs it (with the CPU baseline); its kernel trace and FETCH_SIZE pass (summaries
# for profiles/ and bench.committed_traffic); the other workloads' lines.
set -o pipefail
O=gpurun_out/r04z2; mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-300 $O/bench_default.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kp_attn3" -d $R/$O/pmc -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof/run_results.db --pmc $R/$O/pmc/run_results.db \
  --out $R/$O/r04_complex-fb15k237-sufficient > $R/$O/prof_summary.txt 2>&1 || exit 1
python3 $R/tools/timeline.py $R/$O/prof/run_results.db --window 0.4 --skip-end 0.05 --gaps > $R/$O/timeline_default.txt 2>&1 || exit 1
rm -rf $R/$O/prof $R/$O/pmc
head -8 $R/$O/timeline_default.txt
cd $R
for w in complex-fb15k237-necessary complex-db100k-necessary complex-db100k-sufficient; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  echo "$w $(grep -o '"value": [0-9.]*' $O/bench_$w.json)"
done
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 20 --warmup 3 --no-cpu-baseline \
  > $O/bench_transe-fb15k237-necessary.json 2> $O/bench_transe-fb15k237-necessary.err || exit 1
echo "transe $(grep -o '"value": [0-9.]*' $O/bench_transe-fb15k237-necessary.json)"
timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 --no-cpu-baseline \
  > $O/bench_conve-yago310-necessary.json 2> $O/bench_conve-yago310-necessary.err || exit 1
echo "conve $(grep -o '"value": [0-9.]*' $O/bench_conve-yago310-necessary.json)"
echo done
