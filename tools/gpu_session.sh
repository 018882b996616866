#!/bin/bash
# One GPU session: GPU parity suite -> bench of every config (N = 1) -> PMC passes of every
# config's trace kernel -> rocprofv3 kernel trace of $TRACE_CFGS. Every GPU step has its own
# time limit; the chain stops at the first failure.
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
fi
echo "== bench all" && STEPS=${STEPS:-10} CONFIGS="${BENCH_CFGS:-C1 C2 C3 C4 C5}" bash tools/bench_all.sh || exit 1
if [ -n "$PMC_CFGS" ]; then
  echo "== pmc" && CONFIGS="$PMC_CFGS" bash tools/pmc_all.sh || exit 1
fi
for c in $TRACE_CFGS; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof_$c.json 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; exit 1; }
  python tools/trace_span.py $(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1) --skip 1 || true
done
echo done
