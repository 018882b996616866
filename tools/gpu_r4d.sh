#!/bin/bash
# Round-4 full measurement session: GPU parity suite -> smoke -> default bench line -> rocprofv3
# of the default command -> bench of every config (N = 1) -> PMC -> per-config rocprofv3 traces
# -> the 8-GPU plans' shards -> the N-rank path rehearsed on one GPU (gloo staging).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ -n "$PRE_AB" ]; then  # block-size knob on the C4 plan shard and whole frame
  echo "== ab C4 plan-8 shard 0" && CFG=C4 VARIANTS="$PRE_AB" ROUNDS=2 EXTRA="--no-host-path --plan-gpus 8 --shard 0" bash tools/ab.sh || exit 1
  echo "== ab C4" && CFG=C4 VARIANTS="$PRE_AB" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
  echo "== ab C2" && CFG=C2 VARIANTS="$PRE_AB" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
fi
echo "== default bench" && timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
  || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo "== rocprof default" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- python bench.py > $OUT/bench_default_prof.json 2> $OUT/prof_default.err \
  || { echo "rocprof default failed"; tail -20 $OUT/prof_default.err; exit 1; }
python tools/trace_span.py $(find $OUT/prof_default -name "*kernel_trace.csv" | head -1) --skip 2 > $OUT/trace_span_default.txt || true
cat $OUT/trace_span_default.txt
if [ -z "$SKIP_ALL" ]; then
  echo "== bench all" && STEPS=${STEPS:-10} CONFIGS="${BENCH_CFGS:-C1 C2 C3 C4 C5}" bash tools/bench_all.sh || exit 1
fi
if [ -n "${PMC_CFGS-C2 C3}" ]; then
  echo "== pmc" && CONFIGS="${PMC_CFGS-C2 C3}" bash tools/pmc_all.sh || exit 1
fi
for c in ${TRACE_CFGS-C2 C3 C4 C5}; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof_$c.json 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; exit 1; }
  python tools/trace_span.py $(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1) --skip 1 > $OUT/trace_span_$c.txt || true
  cat $OUT/trace_span_$c.txt
done
if [ -z "$SKIP_PLAN" ]; then
  echo "== plan shards"
  CONFIGS="${PLAN_CFGS:-C2 C4 C5}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
    || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
  python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
fi
for n in ${REHEARSE_N-2 4}; do
  for c in ${REHEARSE_CFGS:-C4 C5}; do
    echo "== rehearsal --gpus $n --config $c (ranks share GPU 0, gloo)"
    BHRT_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus $n --config $c --steps 4 --warmup 1 \
      > $OUT/rehearse_${n}_$c.json 2> $OUT/rehearse_${n}_$c.err \
      || { echo "rehearsal failed"; tail -30 $OUT/rehearse_${n}_$c.err; exit 1; }
    cat $OUT/rehearse_${n}_$c.json
  done
done
echo all-done
