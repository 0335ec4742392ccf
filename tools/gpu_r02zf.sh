set -eo pipefail
# kp_attn3 chained S phase (KP_S_CHAIN): micro A/B against HEAD (bitwise hash + time),
# then every GPU test and the default bench with the new library
O=gpurun_out/r02zf; mkdir -p $O
bash tools/attn_micro.sh run r02zf old chain nochain
python - <<'PY'
import json
rows = {}
for v in ("old", "chain", "nochain"):
    for line in open(f"gpurun_out/r02zf/{v}.jsonl"):
        d = json.loads(line)
        if "ms" in d:
            rows.setdefault((d["DB"], d["mode"], d["n_ent"]), {}).setdefault(v, []).append((d["ms"], d["bits"], d["err_o"]))
bad = 0
for k, r in rows.items():
    bits = {v: {b for _, b, _ in x} for v, x in r.items()}
    same = len(set().union(*bits.values())) == 1
    bad += not same
    print(k, {v: round(min(m for m, _, _ in x), 4) for v, x in r.items()}, "bitwise same" if same else f"DIFF {bits}")
if bad:
    raise SystemExit("variants differ")
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['roofline']['frac'], d['roofline']['device_kernel_ms_per_launch'])"
timeout -k 10 300 python bench.py --workload transe-fb15k237-necessary --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_transe.json 2> $O/bench_transe.err
python -c "import json;d=json.load(open('$O/bench_transe.json'));print('transe', d['value'], d['ms_per_step'])"; grep breakdown $O/bench_transe.err || true
echo done
