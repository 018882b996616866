#!/bin/bash
# bench.py over every BASELINE configuration at N=1 (C1..C5); one JSON line each ($BENCH_ARGS:
# extra bench.py flags).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/bench_all}; mkdir -p $OUT
for c in ${CONFIGS:-C1 C2 C3 C4 C5}; do
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 $BENCH_ARGS > $OUT/$c.json 2> $OUT/$c.err \
    || { echo "$c failed"; tail -5 $OUT/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', d['value'], d['unit'], d['scaling'], d['config']['width'], 'x', d['config']['height'], 'kern', d['kernel']['avg_ms'], 'ms frac', d['roofline']['frac'], 'cpu', d.get('cpu_baseline', {}).get('value'), 'mism', d.get('class_mismatch'), 'dhit', d.get('max_rel_dhit'), 'display', d.get('display_resident', {}).get('mrays_s'))"
done
