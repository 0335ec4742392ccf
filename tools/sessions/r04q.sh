#!/bin/bash
# r04q: the headline's idle gaps at batch boundaries: the pipeline with cyclic garbage
# collection off while batches are in flight (KELPIE_PIPELINE_NOGC=1) against on,
# alternating three times, and a trace of the off form with its gaps listed.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
R=$(pwd)
for i in 1 2 3; do
  for v in 0 1; do
    KELPIE_PIPELINE_NOGC=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_nogc${v}_$i.json 2> $O/bench_nogc${v}_$i.err || exit 1
    echo "nogc=$v $i $(grep -o '"value": [0-9.]*' $O/bench_nogc${v}_$i.json)"
  done
done
export TMPDIR=/tmp
cd /tmp
KELPIE_PIPELINE_NOGC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
python3 $R/tools/timeline.py $R/$O/prof_default/run_results.db --window 0.4 --skip-end 0.05 --gaps > $R/$O/timeline_default.txt 2>&1 || exit 1
rm -rf $R/$O/prof_default
head -14 $R/$O/timeline_default.txt
echo done
