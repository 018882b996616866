#!/bin/bash
# Round-4 closing session: GPU suite, smoke, the default bench line, the same under rocprofv3.
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
echo all-done
