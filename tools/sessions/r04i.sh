#!/bin/bash
# r04i: the one-split kp_cx_contrib (64 registers: fits beside a resident attention wave)
# against the round-3 library, alternating, with a kernel trace (summaries only) and the
# ComplEx GPU parity tests.
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
R=$(pwd)
lib() { case $1 in r03) echo $R/variants/lib_r03.so ;; *) echo $R/kelpie_amd/libkelpie_hip.so ;; esac; }
for i in 1 2; do
  for v in r03 cur; do
    KELPIE_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.json) $(grep -o '"results_sha16": "[0-9a-f]*"' $O/bench_${v}_$i.json)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "complex" --timeout 120 --timeout-method thread > $O/tests_complex.txt 2>&1
echo "complex tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_complex.txt | tail -5
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_cur -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof_cur.log 2>&1 || exit 1
python3 $R/tools/prof_summary.py --stats $R/$O/prof_cur/run_results.db --out $R/$O/cur > /dev/null || exit 1
python3 $R/tools/timeline.py $R/$O/prof_cur/run_results.db > $R/$O/timeline_cur.txt 2>&1 || exit 1
rm -rf $R/$O/prof_cur
head -6 $R/$O/timeline_cur.txt
echo done
