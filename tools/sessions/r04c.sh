#!/bin/bash
# r04c: ComplEx step split (kp_cx_stepq z, kp_cx_prep lane-per-row fp64 scalars,
# kp_cx_contrib merge only) + fp64 ranks for TransE / ConvE: the ComplEx parity tests and
# every full-size fixture, the default bench line A/B against the round-3 build
# (variants/lib_r03.so, alternating), the ConvE parity tests (three train-mode
# dropouts), and the kernel-trace summary of the default bench.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference.py -m gpu -v \
  -k "complex or fullsize" --timeout 120 --timeout-method thread > $O/tests_complex.txt 2>&1
echo "complex+fullsize tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_complex.txt | tail -8
for i in 1 2; do
  for v in r03 new; do
    L=$R/kelpie_amd/libkelpie_hip.so; [ $v = r03 ] && L=$R/variants/lib_r03.so
    KELPIE_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
    cut -c1-200 $O/bench_${v}_$i.json
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "conve" --timeout 120 \
  --timeout-method thread > $O/tests_conve.txt 2>&1
echo "conve tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests_conve.txt | tail -8
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_default.log 2>&1 || exit 1
echo done
