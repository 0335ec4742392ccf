set -o pipefail
O=gpurun_out/${TAG:-s36}; mkdir -p $O
export KP_ATTN=bf16x3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "full_width or vs_reference_goldens" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in complex-fb15k237-sufficient conve-yago310-necessary; do
timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || exit 1
python -c "import json;d=json.load(open('$O/$w.json'));print('$w', round(d['value'],1), round(d['roofline']['avg_launch_ms'],4))"
done
