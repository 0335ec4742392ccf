#!/bin/bash
# One parameterised GPU-box session (replaces the per-session one-off scripts):
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
# Each step is `name[:arg[:arg...]]`; every step runs under its own time limit and the
# session stops at the first failing step.  Output: gpurun_out/<tag>/.
#   smoke                              __graft_entry__.smoke()
#   tests[:<-k expr>]                  pytest -m gpu (optionally -k), verbose, 120 s per test
#   micro:<variant>[:<reps>]           variants/attn_micro_<variant> on the three attention shapes
#   microfb:<variant>[:<reps>]         the same, FB15k-237 ComplEx shape only (microcv: ConvE YAGO3-10 only)
#   pmcmicro:<variant>                 settled-clock counter passes of the micro (FB15k-237 shape)
#   bench:<workload>[:steps[:warmup[:VAR=val,...]]]   one bench line (no CPU baseline)
#   benchcpu                           the default line as the driver runs it (with the CPU baseline)
#   builderab:<VAR>:<v1,..>[:reps[:preds]]  builder leg A/B over an env switch
#   builderprof[:preds]               kernel trace + device timeline of the builder leg
#   prof:<workload>[:steps]            rocprofv3 kernel trace + FETCH_SIZE/WRITE_SIZE passes + summary
#   pmcbench:<workload>:<regex>        SQ counter pass of one bench workload's kernels
#   ab:<workload>:<VAR>:<v1,v2,..>[:reps[:steps]]    alternating env A/B of the bench
#   rehearse:<args>                    tools/sched_rehearsal.py with ','-separated args
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
R=$(pwd)
MICRO_SHAPES=("25 0 14541 3100 30" "25 0 99604 1800 10" "13 2 123182 4270 10")

run_step() {
  local spec=$1
  IFS=':' read -r -a a <<< "$spec"
  local n=${a[0]}
  case $n in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || return 1
      tail -1 $O/smoke.txt ;;
    tests)
      local k=()
      [ -n "${a[1]}" ] && k=(-k "${a[1]}")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "${k[@]}" \
        > $O/tests_${a[1]:-all}.txt 2>&1
      local rc=$?
      grep -E "passed|failed|error" $O/tests_${a[1]:-all}.txt | tail -2
      return $rc ;;
    rngbench)  # the TransE draw chains timed apart on the box's CPU (tools/rng_bench.cpp)
      g++ -O3 -std=c++17 -mavx2 -mfma -ffp-contract=off -pthread -Iinclude tools/rng_bench.cpp -o /tmp/rng_bench_$TAG || return 1
      timeout -k 10 120 /tmp/rng_bench_$TAG ${a[1]:-5} > $O/rng_bench.txt 2>&1 || return 1
      tail -6 $O/rng_bench.txt ;;
    hostprof)  # host scheduling cost of one workload's batches (CPU only)
      timeout -k 10 300 python -u tools/host_profile.py --workload ${a[1]:-transe-fb15k237-necessary} --preds 16 \
        --repeats ${a[2]:-6} > $O/host_profile_${a[1]:-transe-fb15k237-necessary}.txt 2>&1
      local rc=$?
      grep -E "^batch" $O/host_profile_${a[1]:-transe-fb15k237-necessary}.txt || true
      return $rc ;;
    micro|microfb|microdb|microcv)
      local v=${a[1]} reps=${a[2]:-2} envs=() tagx=""
      if [ -n "${a[3]}" ]; then IFS=',' read -r -a envs <<< "${a[3]}"; tagx="_$(echo ${a[3]} | tr ',=' '__')"; fi
      local shapes=("${MICRO_SHAPES[@]}")
      [ $n = microfb ] && shapes=("${MICRO_SHAPES[0]}")
      [ $n = microdb ] && shapes=("${MICRO_SHAPES[0]}" "${MICRO_SHAPES[1]}")
      [ $n = microcv ] && shapes=("${MICRO_SHAPES[2]}")
      for rep in $(seq 1 $reps); do
        for args in "${shapes[@]}"; do
          env "${envs[@]}" timeout -k 10 120 variants/attn_micro_$v $args 0.05 >> $O/micro_$v$tagx.jsonl || return 1
        done
      done
      grep -v stamps $O/micro_$v$tagx.jsonl | cut -c1-260 | tail -$(( reps * ${#shapes[@]} )) || true
      grep stamps $O/micro_$v$tagx.jsonl | tail -2 || true ;;
    pmcmicro)
      # pmcmicro:<variant>[:<envs>[:<shape index into MICRO_SHAPES, default 0 = ComplEx FB15k-237>]]
      local v=${a[1]} i=0 envs=() si=${a[3]:-0}
      [ -n "${a[2]}" ] && IFS=',' read -r -a envs <<< "${a[2]}"
      for e in "${envs[@]}"; do export "$e"; done
      export TMPDIR=/tmp
      for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
               "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum" \
               "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"; do
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -d $R/$O/pmc_${v}_s${si}_p$i -o run -- \
          $R/variants/attn_micro_$v ${MICRO_SHAPES[$si]} 0.05 > $R/$O/pmc_${v}_s${si}_p$i.log 2>&1) || return 1
        python3 tools/pmc_dump.py $O/pmc_${v}_s${si}_p$i/run_results.db kp_attn >> $O/pmc_${v}_s$si.txt 2>&1 || return 1
        rm -rf $O/pmc_${v}_s${si}_p$i
        i=$((i + 1))
      done
      cat $O/pmc_${v}_s$si.txt ;;
    bench)
      local w=${a[1]} st=${a[2]:-3} wu=${a[3]:-1} envs=() tagx=""
      if [ -n "${a[4]}" ]; then IFS=',' read -r -a envs <<< "${a[4]}"; tagx="_$(echo ${a[4]} | tr ',=/' '___')"; fi
      env "${envs[@]}" timeout -k 10 600 python bench.py --workload $w --steps $st --warmup $wu --no-cpu-baseline --builder-preds 0 \
        > $O/bench_$w$tagx.json 2> $O/bench_$w$tagx.err || { tail -5 $O/bench_$w$tagx.err; return 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value'],1), 'cand/s', round(d['ms_per_step'],2), 'ms', 'frac', d['roofline']['frac'], 'fp64', d.get('rank_delta_match_rate_ref_fp64'))" $O/bench_$w$tagx.json "$w$tagx" ;;
    benchcpu)
      timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || return 1
      cut -c1-400 $O/bench_default.json ;;
    builderab)
      # builderab:<VAR>:<v1,v2,..>[:reps[:preds]]: the default line's builder leg, alternating env values
      local var=${a[1]} reps=${a[3]:-2} np=${a[4]:-4}
      IFS=',' read -r -a vals <<< "${a[2]}"
      for rep in $(seq 1 $reps); do
        for v in "${vals[@]}"; do
          env "$var=$v" timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --builder-preds $np \
            > $O/builderab_${var}_${v}_$rep.json 2> $O/builderab_${var}_${v}_$rep.err || { tail -5 $O/builderab_${var}_${v}_$rep.err; return 1; }
          python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);b=d['builder'];print(sys.argv[2], round(b['value'],1), 'rel/s', b['relevances'], 'rel', b['evaluated'], 'eval', b['engine_batches'], 'batches', b.get('time_split_s'), {k: v['#relevances_equal'] and v['top10_rules_equal'] for k, v in b.get('reference_match_first_prediction', {}).items() if k != 'fixture'})" $O/builderab_${var}_${v}_$rep.json "$var=$v"
        done
      done ;;
    builderprof)
      # builderprof[:<preds>]: kernel trace of the default line's builder leg (the run's last kernels)
      local np=${a[1]:-4}
      export TMPDIR=/tmp
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/bprof -o run -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --builder-preds $np > $R/$O/bprof.json 2> $R/$O/bprof.err) || return 1
      local win=$(python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['builder']['execution_time_s'])" $O/bprof.json)
      python3 tools/timeline.py $O/bprof/run_results.db --window $win --skip-end 0 --gaps > $O/builder_timeline.txt 2>&1
      rm -rf $O/bprof
      head -30 $O/builder_timeline.txt ;;
    prof)
      local w=${a[1]} st=${a[2]:-5}
      export TMPDIR=/tmp
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$w -o run -- \
        python3 $R/bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline --builder-preds 0 > $R/$O/prof_$w.log 2>&1) || return 1
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmcf_$w -o run -- \
        python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --builder-preds 0 > $R/$O/pmcf_$w.log 2>&1) || return 1
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmcw_$w -o run -- \
        python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --builder-preds 0 > $R/$O/pmcw_$w.log 2>&1) || return 1
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS \
        -d $R/$O/pmcq_$w -o run -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --builder-preds 0 > $R/$O/pmcq_$w.log 2>&1) || return 1
      python3 tools/prof_summary.py --stats $O/prof_$w/run_results.db --pmc $O/pmcf_$w/run_results.db \
        --pmc-write $O/pmcw_$w/run_results.db --pmc-sq $O/pmcq_$w/run_results.db --out $O/${TAG}_$w > $O/prof_summary_$w.txt 2>&1 || return 1
      python3 tools/timeline.py $O/prof_$w/run_results.db --window 0.4 --skip-end 0.05 --gaps > $O/timeline_$w.txt 2>&1
      rm -rf $O/prof_$w $O/pmcf_$w $O/pmcw_$w $O/pmcq_$w
      head -20 $O/prof_summary_$w.txt ;;
    pmcbench)
      local w=${a[1]} rx=${a[2]}
      export TMPDIR=/tmp
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
        --kernel-include-regex "$rx" -d $R/$O/pmcs_$w -o run -- \
        python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --builder-preds 0 > $R/$O/pmcs_$w.log 2>&1) || return 1
      python3 tools/pmc_dump.py $O/pmcs_$w/run_results.db "$rx" > $O/pmcs_$w.txt 2>&1
      rm -rf $O/pmcs_$w
      cat $O/pmcs_$w.txt ;;
    ab)
      local w=${a[1]} var=${a[2]} reps=${a[4]:-2} st=${a[5]:-3}
      IFS=',' read -r -a vals <<< "${a[3]}"
      for rep in $(seq 1 $reps); do
        for v in "${vals[@]}"; do
          run_step "bench:$w:$st:1:$var=$v" || return 1
          mv $O/bench_${w}_${var}_$v.json $O/ab_${w}_${var}_${v}_$rep.json
        done
      done ;;
    libab)  # libab:<wl>:<base|variant,...>[:reps[:steps]]: variants/lib_<variant>.so against the product library
      local w=${a[1]} reps=${a[3]:-2} st=${a[4]:-3}
      IFS=',' read -r -a vals <<< "${a[2]}"
      for rep in $(seq 1 $reps); do
        for v in "${vals[@]}"; do
          local lib=$R/kelpie_amd/libkelpie_hip.so
          [ $v != base ] && lib=$R/variants/lib_$v.so
          KELPIE_HIP_LIB=$lib timeout -k 10 600 python bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline --builder-preds 0 \
            > $O/libab_${w}_${v}_$rep.json 2> $O/libab_${w}_${v}_$rep.err || { tail -5 $O/libab_${w}_${v}_$rep.err; return 1; }
          python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value'],1), 'cand/s', round(d['ms_per_step'],2), 'ms', 'frac', d['roofline']['frac'], 'fp64', d.get('rank_delta_match_rate_ref_fp64'))" $O/libab_${w}_${v}_$rep.json "$w $v"
        done
      done ;;
    fullsize)
      timeout -k 10 900 python tools/fullsize_table.py $(echo ${a[1]} | tr ',' ' ') > $O/fullsize_table.jsonl 2> $O/fullsize_table.err || { tail -3 $O/fullsize_table.err; return 1; }
      cut -c1-400 $O/fullsize_table.jsonl ;;
    rehearse)
      timeout -k 10 900 python tools/sched_rehearsal.py $(echo ${a[1]} | tr ',' ' ') > $O/rehearse_${a[1]//,/_}.txt 2>&1 || return 1
      tail -5 $O/rehearse_${a[1]//,/_}.txt ;;
    *)
      echo "unknown step $spec"; return 1 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  run_step "$s" || { echo "step $s failed"; exit 1; }
done
echo "session $TAG done"
