set -eo pipefail
O=gpurun_out/r02o; mkdir -p $O
for nq in 800 1600 3100 5000; do for part in 1 2; do
  timeout -k 10 120 variants/attn_micro_cur 25 0 14541 $nq 20 0.05 $part >> $O/part.jsonl
done; done
timeout -k 10 600 python -u -m pytest tests/test_verification.py -m gpu -v --timeout 240 --timeout-method thread > $O/verify_tests.log 2>&1 || { tail -40 $O/verify_tests.log; exit 1; }
tail -3 $O/verify_tests.log
timeout -k 10 600 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 > $O/bench_conve.json 2> $O/bench_conve.err
cat $O/bench_conve.json
