#!/bin/bash
# Round-4 final refresh after the Kerr-path SALU changes (bit-identical): GPU suite, smoke,
# default bench line, bench of every config, PMC of C2/C4/C5, traces of C4/C5, C4 plan shards.
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
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['kernel']['avg_ms'], d['roofline']['frac'], d['host_path']['trace_rays_batch_mrays_s'], d['host_path']['trace_rays_batch_after_frames_mrays_s'])"
echo "== bench all" && STEPS=10 bash tools/bench_all.sh || exit 1
echo "== pmc" && CONFIGS="C2 C4 C5" bash tools/pmc_all.sh || exit 1
for c in C4 C5; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof_$c.json 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; exit 1; }
  python tools/trace_span.py $(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1) --skip 1 > $OUT/trace_span_$c.txt || true
  cat $OUT/trace_span_$c.txt
done
echo "== plan shards C4"
CONFIGS="C4" bash tools/plan_shards.sh > $OUT/plan_shards_c4.jsonl 2> $OUT/plan_shards.err \
  || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
python tools/plan_summary.py $OUT/plan_shards_c4.jsonl --out $OUT/plan_summary_c4.txt
echo all-done
