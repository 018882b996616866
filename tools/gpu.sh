#!/bin/bash
# The one GPU-session runner (replaces the per-session tools/gpu_r*.sh scripts of rounds 3-4).
# Runs the named steps in order on the GPU box; every GPU step has its own time limit and the
# chain stops at the first failure (a fault, an abort or a time limit ends the session there).
#
#   tools/gpu.sh STEP [STEP ...]
#
# Steps (outputs under gpurun_out/$TAG, TAG defaults to "s"):
#   tests          python -m pytest tests -m gpu (-x, per-test timeout)
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (bench.py, no flags)
#   rocprof        the default bench line under rocprofv3 --kernel-trace --stats (+ trace span)
#   rocprof_timed  the timed frames alone under rocprofv3: busy span per dispatch vs the line's avg_ms
#   bench_all      bench.py --config C1..C5 ($CONFIGS), N = 1
#   plan           every shard of the 8-GPU plans of $PLAN_CFGS (tools/plan_shards.sh) + summary
#   pmc            rocprofv3 PMC passes of $PMC_CFGS (tools/pmc_all.sh)
#   ab             interleaved A/B of $VARIANTS on $AB_CFGS (tools/ab.sh; $ROUNDS rounds)
#   ab_tests       the GPU parity suite against each build in $TEST_VARIANTS
#   stamps         per-wave stamps of $STAMP_RUNS ("CFG:PLAN:SHARD:STREAMS ...") with the
#                  diagnostic build diag/libbhrt_stamps.so (tools/wave_stamps.py)
#   steps          per-ray step maps of C2, C4, C5 (tools/dump_steps.py)
#   cmd            run $CMD (one extra command, under a 600 s limit)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fail() { echo "FAILED: $1"; [ -n "$2" ] && tail -n ${3:-30} "$2"; exit 1; }
for step in "$@"; do
  echo "== $step ($(date +%T))"
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || fail tests $OUT/pytest_gpu.log 40
    tail -n 1 $OUT/pytest_gpu.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
      || fail smoke $OUT/smoke.log
    tail -n 1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 400 python bench.py $BENCH_ARGS > $OUT/bench_default.json 2> $OUT/bench_default.err \
      || fail bench $OUT/bench_default.err
    cat $OUT/bench_default.json ;;
  rocprof)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv \
      -- python bench.py $BENCH_ARGS > $OUT/bench_default_prof.json 2> $OUT/prof_default.err \
      || fail rocprof $OUT/prof_default.err
    python tools/trace_span.py $(find $OUT/prof_default -name "*kernel_trace.csv" | head -1) --skip 2 \
      > $OUT/trace_span_default.txt || true
    cat $OUT/trace_span_default.txt ;;
  rocprof_timed)
    # like-for-like: the timed frames only (no extra legs), their busy span per dispatch from the
    # trace against the profiled line's own kernel.avg_ms
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_timed -o run --output-format csv \
      -- python bench.py --no-host-path --no-cpu-baseline --steps ${STEPS:-20} $BENCH_ARGS > $OUT/bench_timed_prof.json \
      2> $OUT/prof_timed.err || fail rocprof_timed $OUT/prof_timed.err
    python tools/trace_span.py $(find $OUT/prof_timed -name "*kernel_trace.csv" | head -1) --last ${STEPS:-20} \
      > $OUT/trace_span_timed.txt || true
    cat $OUT/trace_span_timed.txt
    python3 -c "import json; d=json.load(open('$OUT/bench_timed_prof.json')); print('profiled line kernel.avg_ms', d['kernel']['avg_ms'], 'value', d['value'])" ;;
  bench_all)
    OUT=$OUT/bench_all STEPS=${STEPS:-10} CONFIGS="${CONFIGS:-C1 C2 C3 C4 C5}" bash tools/bench_all.sh \
      || fail bench_all ;;
  plan)
    STEPS=${STEPS:-20} CONFIGS="${PLAN_CFGS:-C2 C4 C5}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl \
      2> $OUT/plan_shards.err || fail plan $OUT/plan_shards.err
    python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt && cat $OUT/plan_summary.txt ;;
  pmc)
    CONFIGS="${PMC_CFGS:-C2 C3 C4 C5}" bash tools/pmc_all.sh || fail pmc
    mkdir -p $OUT/pmc && mv gpurun_out/pmc_C*.json $OUT/pmc/ 2>/dev/null; true ;;
  ab)
    for cfg in ${AB_CFGS:-C2}; do
      CFG=$cfg VARIANTS="${VARIANTS:-base}" ROUNDS=${ROUNDS:-3} bash tools/ab.sh > $OUT/ab_$cfg.txt 2>&1 \
        || fail "ab $cfg" $OUT/ab_$cfg.txt
      cat $OUT/ab_$cfg.txt
    done ;;
  ab_tests)
    for v in $TEST_VARIANTS; do
      BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu \
        -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || fail "ab_tests $v" $OUT/pytest_$v.log
      echo "$v: $(tail -n 1 $OUT/pytest_$v.log)"
    done ;;
  stamps)
    for run in ${STAMP_RUNS:-C4:8:0:4 C4:1:0:2}; do
      IFS=: read cfg plan shard streams <<< "$run"
      f=$OUT/stamps_${cfg}_p${plan}_s${shard}_x${streams}.npz
      BHRT_LIB=raytracing-engine-in-c_amd/diag/libbhrt_stamps.so timeout -k 10 300 python tools/wave_stamps.py \
        --config $cfg --plan-gpus $plan --shard $shard --streams $streams --frames ${FRAMES:-20} --out $f \
        > $OUT/stamps.log 2>&1 || fail stamps $OUT/stamps.log
      python tools/wave_stamps.py --analyse $f
    done ;;
  steps)
    timeout -k 10 300 python tools/dump_steps.py --out $OUT/steps.npz > $OUT/steps.log 2>&1 || fail steps $OUT/steps.log
    cat $OUT/steps.log ;;
  cmd)
    timeout -k 10 600 bash -c "$CMD" > $OUT/cmd.log 2>&1 || fail cmd $OUT/cmd.log
    tail -n 40 $OUT/cmd.log ;;
  *) fail "unknown step $step" ;;
  esac
done
echo "all steps done ($(date +%T))"
