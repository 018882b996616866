#!/bin/bash
# Round-4 session E: frames in flight on the C4 8-GPU-plan shard with libbhrt's streams created
# lazily and 8 hardware queues (bench.py): stream sweep, then the C4 and C2 plan shards.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for st in ${STREAM_SWEEP-2 3 4}; do
  for ex in "--plan-gpus 8 --shard 0" ""; do
    timeout -k 10 120 python bench.py --config C4 --steps 40 --warmup 4 --no-cpu-baseline --no-host-path --streams $st $ex > $OUT/c4_streams.json 2>/dev/null \
      || { echo "streams $st failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_streams.json')); print('C4 streams $st', '$ex', d['value'], d['ms_per_step'], 'host', d['kernel']['host_issue_ms_per_step'])"
  done
done
echo "== rocprof C4 plan shard"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C4_p8e -o run --output-format csv -- python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --plan-gpus 8 --shard 0 > $OUT/bench_prof_C4_p8e.json 2> $OUT/prof_C4_p8e.err \
  || { echo "rocprof failed"; tail -20 $OUT/prof_C4_p8e.err; exit 1; }
python tools/frame_timeline.py $(find $OUT/prof_C4_p8e -name "*kernel_trace.csv" | head -1) --skip 3 || true
if [ -z "$SKIP_PLAN" ]; then
  echo "== plan shards"
  CONFIGS="${PLAN_CFGS:-C4 C2}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
    || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
  python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
fi
echo all-done
