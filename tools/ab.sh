#!/bin/bash
# A/B of libbhrt build variants on the bench workload (two interleaved rounds).
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab; mkdir -p $OUT
CFG=${CFG:-C2}
VARIANTS=${VARIANTS:-"base w4 fs fsw4 w5 ctr"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    if [ "$v" = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$v.so; fi
    BHRT_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline $EXTRA > $OUT/${v}_$round.json 2>$OUT/${v}_$round.err || { echo "$v failed"; tail -3 $OUT/${v}_$round.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$round.json')); print('$v', $round, d['value'], d['kernel']['avg_ms'])"
  done
done
