#!/bin/bash
# Round-4 session F: with 8 hardware queues per process, 4 frames in flight (--streams 4)
# against 2 on every config's N = 1 line and on the 8-GPU plan shards of C2, C4 and C5 (every
# stream warmed: bench.py runs at least one untimed frame per stream).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in C1 C2 C3 C4 C5; do
  for st in 2 4 2 4; do
    timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --streams $st > $OUT/f_n1.json 2>/dev/null \
      || { echo "$cfg streams $st failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/f_n1.json')); print('$cfg N=1 streams $st', d['value'], d['ms_per_step'])"
  done
done
echo "== plan shards, --streams 4"
WARMUP=4 BENCH_ARGS="--streams 4" CONFIGS="C4 C2 C5" bash tools/plan_shards.sh > $OUT/plan_shards_s4.jsonl 2> $OUT/plan_shards_s4.err \
  || { echo "plan shards failed"; tail -20 $OUT/plan_shards_s4.err; exit 1; }
python tools/plan_summary.py $OUT/plan_shards_s4.jsonl --out $OUT/plan_summary_s4.txt
echo all-done
