set -eo pipefail
# register-row panel with DPP argmax: parity tests, bitwise comparison with the unblocked kernel, timing, stamps
O=gpurun_out/r02u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_baselines.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
KELPIE_HIP_LIB=$PWD/variants/lib_crold.so timeout -k 10 300 python tools/baselines_bench.py --preds 16 --dump $O/criage_old.npy > $O/bench_old.jsonl 2> $O/bench_old.err
for v in main seg16; do
  if [ $v = main ]; then L=$PWD/kelpie_amd/libkelpie_hip.so; else L=$PWD/variants/lib_$v.so; fi
  KELPIE_HIP_LIB=$L timeout -k 10 300 python tools/baselines_bench.py --preds 16 --dump $O/criage_$v.npy > $O/bench_$v.jsonl 2> $O/bench_$v.err
  KELPIE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python tools/baselines_bench.py --preds 16 > $O/prof_$v.log 2>&1
  python -c "
import numpy as np, json
a=np.load('$O/criage_$v.npy'); b=np.load('$O/criage_old.npy')
d=json.loads(open('$O/bench_$v.jsonl').read().splitlines()[1])
print('$v', 'n', a.size, 'bitwise equal to unblocked', np.array_equal(a.view(np.int64), b.view(np.int64)), 'cand/s', round(d['value']))
"
done
KELPIE_HIP_LIB=$PWD/variants/lib_crst.so timeout -k 10 300 python tools/baselines_bench.py --preds 16 > $O/st.log 2>&1
grep "cr stamps" $O/st.log | head -3
