#!/bin/bash
# r04x: ConvE YAGO3-10 with three batches in flight against two (KELPIE_PIPELINE_DEPTH),
# alternating twice, and a ConvE trace with its idle gaps listed.
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
R=$(pwd)
for i in 1 2; do
  for d in 2 3; do
    KELPIE_PIPELINE_DEPTH=$d timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 4 --warmup 1 \
      --no-cpu-baseline > $O/bench_conve_depth${d}_$i.json 2> $O/bench_conve_depth${d}_$i.err || exit 1
    echo "depth=$d $i $(grep -o '"value": [0-9.]*' $O/bench_conve_depth${d}_$i.json)"
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_conve -o run -- \
  python3 $R/bench.py --workload conve-yago310-necessary --steps 6 --warmup 1 --no-cpu-baseline > $R/$O/prof_conve.log 2>&1 || exit 1
python3 $R/tools/timeline.py $R/$O/prof_conve/run_results.db --kernel "kp_attn3<13" --window 1.2 --skip-end 0.05 --gaps \
  > $R/$O/timeline_conve.txt 2>&1 || exit 1
rm -rf $R/$O/prof_conve
head -16 $R/$O/timeline_conve.txt
echo done
