#!/bin/bash
# k_trace refill threshold sweep on one config (CFG, default C4): kernel ms per threshold.
cd "$(dirname "$0")/.."
OUT=gpurun_out/refill; mkdir -p $OUT
CFG=${CFG:-C4}
for t in ${THRESHOLDS:-4 8 16 24 32}; do
  timeout -k 10 300 python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --refill $t \
    > $OUT/${CFG}_$t.json 2>$OUT/${CFG}_$t.err || { echo "refill $t failed"; tail -3 $OUT/${CFG}_$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${CFG}_$t.json')); print('$CFG refill $t', d['value'], d['kernel']['avg_ms'])"
done
