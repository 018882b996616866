#!/bin/bash
# Same-box A/B of bench.py --streams S for S in $STREAMS (default 1 2: frames on one stream vs
# alternating streams).
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab_streams; mkdir -p $OUT
for cfg in ${CFGS:-C2 C4}; do
  for round in $(seq 1 ${ROUNDS:-3}); do
    for s in ${STREAMS:-1 2}; do
      timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --streams $s --no-cpu-baseline --no-host-path > $OUT/${cfg}_s${s}_$round.json 2>$OUT/${cfg}_s${s}_$round.err || { echo "$cfg s$s failed"; tail -3 $OUT/${cfg}_s${s}_$round.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${cfg}_s${s}_$round.json')); print('$cfg', 'streams $s', $round, d['value'], 'ms/step', d['ms_per_step'], 'kern', d['kernel']['avg_ms'], 'frac', d['roofline']['frac'])"
    done
  done
done
