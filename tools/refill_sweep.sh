#!/bin/bash
# Refill-threshold sweep: CONFIGS="C2 C4" REFILLS="0 4 8 16" (0 = the per-scene default), 2 rounds.
cd "$(dirname "$0")/.."
OUT=gpurun_out/refill; mkdir -p $OUT
for round in 1 2; do
  for cfg in ${CONFIGS:-C2}; do
    for r in ${REFILLS:-0 4 8 16 32}; do
      a=""; [ "$r" != 0 ] && a="--refill $r"
      timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-host-path $a > $OUT/${cfg}_${r}_${round}.json 2>$OUT/${cfg}_${r}_$round.err || { echo "$cfg $r failed"; tail -3 $OUT/${cfg}_${r}_$round.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${cfg}_${r}_${round}.json')); print('$cfg', 'refill', '$r', $round, d['value'], d['kernel']['avg_ms'])"
    done
  done
done
