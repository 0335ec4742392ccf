set -eo pipefail
# ConvE FC GEMMs on wide tiles: bitwise equality with the previous build, ConvE parity tests, bench, kernel stats
O=gpurun_out/r02x; mkdir -p $O
export TMPDIR=/tmp
KELPIE_HIP_LIB=$PWD/variants/lib_fcold.so timeout -k 10 300 python tools/conve_bitwise.py $O/old.npy > $O/bw_old.log 2>&1
timeout -k 10 300 python tools/conve_bitwise.py $O/new.npy > $O/bw_new.log 2>&1
python -c "
import numpy as np
a=np.load('$O/new.npy'); b=np.load('$O/old.npy')
print('conve relevances', a.size, 'bitwise equal', np.array_equal(a.view(np.int64), b.view(np.int64)))
"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "conve or ConvE" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_conve.json 2> $O/bench_conve.err
cat $O/bench_conve.json | head -c 400; echo
bash tools/kstats.sh $O conve-yago310-necessary 2
