#!/bin/bash
# Round-4 final measurement, part A: GPU parity suite -> smoke -> default bench line -> the same
# command under rocprofv3 (kernel stats + trace span) -> bench of every config (N = 1) -> PMC of
# C2 and C3 (C4/C5 kernels unchanged since profiles/pmc_C4.json, pmc_C5.json).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo "== default bench" && timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
  || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo "== rocprof default" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- python bench.py > $OUT/bench_default_prof.json 2> $OUT/prof_default.err \
  || { echo "rocprof default failed"; tail -20 $OUT/prof_default.err; exit 1; }
python tools/trace_span.py $(find $OUT/prof_default -name "*kernel_trace.csv" | head -1) --skip 2 > $OUT/trace_span_default.txt || true
cat $OUT/trace_span_default.txt
echo "== bench all" && STEPS=10 bash tools/bench_all.sh || exit 1
echo "== pmc" && CONFIGS="C2 C3" bash tools/pmc_all.sh || exit 1
echo all-done
