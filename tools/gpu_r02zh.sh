set -eo pipefail
# ConvE FC GEMMs on bf16x3 MFMA (kp_gemm3_abt, split images of the weights): every GPU test,
# against the fp32 kp_gemm_abt (KP_FC=f32), alternating, and the kernel summary
O=gpurun_out/r02zh; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in both f32 fwd bwd both f32; do
  export KP_FC=$m
  timeout -k 10 600 python bench.py --workload conve-yago310-necessary --steps 3 --warmup 1 --no-cpu-baseline > $O/c_$m.json 2> $O/c_$m.err
  python -c "import json;d=json.load(open('$O/c_$m.json'));print('$m', round(d['value'],1), round(d['ms_per_step'],1), d.get('rank_delta_match_rate'), d['roofline']['frac'])"
done
unset KP_FC
bash tools/kstats.sh $O conve-yago310-necessary 3
echo done
