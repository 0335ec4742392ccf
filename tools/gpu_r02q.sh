set -eo pipefail
# blocked CRIAGE elimination: parity tests, old-vs-new bitwise comparison, before/after kernel stats
O=gpurun_out/r02q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_baselines.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/baselines_bench.py --preds 16 --dump $O/criage_new.npy > $O/bench_new.jsonl 2> $O/bench_new.err
KELPIE_HIP_LIB=$PWD/variants/lib_crold.so timeout -k 10 300 python tools/baselines_bench.py --preds 16 --dump $O/criage_old.npy > $O/bench_old.jsonl 2> $O/bench_old.err
cat $O/bench_new.jsonl $O/bench_old.jsonl
python -c "
import numpy as np
a=np.load('$O/criage_new.npy'); b=np.load('$O/criage_old.npy')
print('n', a.size, 'bitwise equal', np.array_equal(a.view(np.int64), b.view(np.int64)), 'nan', int(np.isnan(a).sum()), 'max rel', float(np.nanmax(np.abs(a-b)/np.maximum(np.abs(b),1e-300))))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run -- python tools/baselines_bench.py --preds 16 > $O/prof_new.log 2>&1
KELPIE_HIP_LIB=$PWD/variants/lib_crold.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_old -o run -- python tools/baselines_bench.py --preds 16 > $O/prof_old.log 2>&1
find $O -name "*kernel_stats.csv" | head
