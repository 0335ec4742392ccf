set -eo pipefail
O=gpurun_out/r02e; mkdir -p $O
cp profiles/conditioning_complex-db100k-necessary.json $O/cond_db100k.json
timeout -k 10 300 python tools/gpu_sample.py $O/cond_db100k.json gpu_centred > $O/sample_centred.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 3 > $O/bench_conve.json 2> $O/bench_conve.err
