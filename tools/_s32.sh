set -o pipefail
O=gpurun_out/${TAG:-s33}; mkdir -p $O
export KP_ATTN=bf16x3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "full_width or all_scores or vs_reference_goldens or db100k or deterministic" > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/suf.json 2> $O/suf.err && cat $O/suf.json || { tail -5 $O/suf.err; exit 1; }
timeout -k 10 300 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/conve.json 2> $O/conve.err && cat $O/conve.json
