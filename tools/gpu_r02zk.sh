set -eo pipefail
# ConvE bf16x3 FC GEMMs with one LDS stage (KP_FC_STAGES=1: four workgroups per CU): the
# ConvE GPU tests on that path, then the ConvE bench against fp32, alternating
O=gpurun_out/r02zk; mkdir -p $O
KP_FC=both KP_FC_STAGES=1 timeout -k 10 600 python -u -m pytest tests -m gpu -k "conve or yago" -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
export KP_FC_STAGES=1
for m in f32 both fwd bwd f32 both; do
  export KP_FC=$m
  timeout -k 10 600 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/c_$m.json 2> $O/c_$m.err
  python -c "import json;d=json.load(open('$O/c_$m.json'));print('$m', round(d['value'],1), round(d['ms_per_step'],1), d.get('rank_delta_match_rate'), d['roofline']['frac'])"
done
echo done
