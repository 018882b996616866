#!/bin/bash
# Round-4 final measurement, part B: per-config rocprofv3 traces, the 8-GPU plans' shards
# (C2, C4, C5), trace_rays_batch, and the N-rank path rehearsed on one GPU (gloo staging).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for c in C2 C3 C4 C5; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof_$c.json 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; exit 1; }
  python tools/trace_span.py $(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1) --skip 1 > $OUT/trace_span_$c.txt || true
  cat $OUT/trace_span_$c.txt
done
echo "== plan shards"
CONFIGS="C2 C4 C5" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
  || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
echo "== batch"
for r in 1 2 3; do
  CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2>/dev/null || { echo "probe failed"; exit 1; }
  head -1 $OUT/bp.txt
done
for n in 2 4; do
  for c in C4 C5; do
    echo "== rehearsal --gpus $n --config $c (ranks share GPU 0, gloo)"
    BHRT_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus $n --config $c --steps 4 --warmup 1 \
      > $OUT/rehearse_${n}_$c.json 2> $OUT/rehearse_${n}_$c.err \
      || { echo "rehearsal failed"; tail -30 $OUT/rehearse_${n}_$c.err; exit 1; }
    cat $OUT/rehearse_${n}_$c.json
  done
done
echo all-done
