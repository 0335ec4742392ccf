#!/bin/bash
# r04a: the ComplEx step split (kp_cx_stepq z, kp_cx_prep lane-per-row fp64 scalars,
# kp_cx_contrib merge only): ComplEx GPU parity + full-size fixtures, then the default
# bench line A/B against the round-3 build (variants/lib_r03.so), alternating, and the
# kernel-trace summary of the new build.
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -x -v \
  -k "complex or fullsize" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  for v in r03 new; do
    L=$R/kelpie_amd/libkelpie_hip.so; [ $v = r03 ] && L=$R/variants/lib_r03.so
    KELPIE_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    cut -c1-200 $O/bench_${v}_$i.json
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
echo done
