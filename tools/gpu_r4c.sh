#!/bin/bash
# Round-4 session C: same-box A/B of claim-schedule knobs on C4 (whole frame and one shard of
# the 8-GPU plan) and C5, then the C4 plan shards with the chosen defaults.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
KNOBS=${KNOBS:-"base base:BHRT_TILE_SCATTER=1 base:BHRT_REFILL=32 base:BHRT_REFILL=48 base:BHRT_QUEUES=4 base:BHRT_QUEUES=32 base:BHRT_CLAIM_MIN=128"}
echo "== ab C4 plan-8 shard 0" && CFG=C4 VARIANTS="$KNOBS" ROUNDS=${AB_ROUNDS:-2} EXTRA="--no-host-path --plan-gpus 8 --shard 0" bash tools/ab.sh || exit 1
echo "== ab C4" && CFG=C4 VARIANTS="$KNOBS" ROUNDS=${AB_ROUNDS:-2} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
[ -z "$C5_KNOBS" ] || { echo "== ab C5" && CFG=C5 VARIANTS="$C5_KNOBS" ROUNDS=${AB_ROUNDS:-2} EXTRA="--no-host-path" bash tools/ab.sh || exit 1; }
for st in ${STREAM_SWEEP-2 3 4}; do  # frames in flight on a C4 plan shard and the whole C4 frame
  for ex in "--plan-gpus 8 --shard 0" ""; do
    timeout -k 10 120 python bench.py --config C4 --steps 40 --warmup 4 --no-cpu-baseline --no-host-path --streams $st $ex > $OUT/c4_streams.json 2>/dev/null \
      || { echo "streams $st failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_streams.json')); print('C4 streams $st', '$ex', d['value'], d['ms_per_step'], 'host', d['kernel']['host_issue_ms_per_step'])"
  done
done
if [ -z "$SKIP_BATCH" ]; then
  for bs in 4 2; do
    echo "== batch probe, $bs trace streams"
    CHUNKS="4 6 8" BHRT_BATCH_STREAMS=$bs BHRT_HOST_TIMING=1 timeout -k 10 300 python tools/batch_probe.py > $OUT/batch_probe_s$bs.txt 2> $OUT/batch_probe_s$bs.err \
      || { echo "batch probe failed"; tail -20 $OUT/batch_probe_s$bs.err; exit 1; }
    cat $OUT/batch_probe_s$bs.txt
  done
fi
if [ -z "$SKIP_PLAN" ]; then
  echo "== plan shards"
  CONFIGS="${PLAN_CFGS:-C4}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
    || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
  python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
fi
echo all-done
