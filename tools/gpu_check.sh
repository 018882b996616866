#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err \
&& echo "== rocprof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof.json 2> $OUT/prof.err
rc=$?
echo "exit=$rc"
tail -3 $OUT/smoke.log $OUT/pytest_gpu.log 2>/dev/null
cat $OUT/bench.json 2>/dev/null
# per-launch GPU time of the overlapping trace launches in the kernel trace (warm-up skipped)
python tools/trace_span.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) --skip 1 2>/dev/null
exit $rc
