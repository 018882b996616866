#!/bin/bash
# Full measurement session for one kernel version: GPU parity suite -> smoke -> default bench
# line -> rocprofv3 trace of the default command -> bench of every config (N = 1) -> PMC of
# every config's trace kernel -> rocprofv3 traces per config. Every GPU step has its own time
# limit; the chain stops at the first failure. Skip parts with SKIP_TESTS / SKIP_ALL / PMC_CFGS="".
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
echo "== default bench" && timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
  || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo "== rocprof default" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- python bench.py > $OUT/bench_default_prof.json 2> $OUT/prof_default.err \
  || { echo "rocprof default failed"; tail -20 $OUT/prof_default.err; exit 1; }
if [ -z "$SKIP_ALL" ]; then
  echo "== bench all" && STEPS=${STEPS:-10} CONFIGS="${BENCH_CFGS:-C1 C2 C3 C4 C5}" bash tools/bench_all.sh || exit 1
fi
if [ -n "${PMC_CFGS-C2 C3 C4 C5}" ]; then
  echo "== pmc" && CONFIGS="${PMC_CFGS-C2 C3 C4 C5}" bash tools/pmc_all.sh || exit 1
fi
for c in ${TRACE_CFGS-C2 C3 C4 C5}; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof_$c.json 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; exit 1; }
  python tools/trace_span.py $(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1) --skip 1 > $OUT/trace_span_$c.txt || true
  cat $OUT/trace_span_$c.txt
done
echo all-done
[ -z "$AB_VARIANTS" ] || bash tools/ab_session.sh || exit 1
