#!/bin/bash
# A/B of library variants on several configs: CONFIGS="C4 C5" VARIANTS="base prev" (2 rounds).
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab; mkdir -p $OUT
for round in 1 2; do
  for cfg in ${CONFIGS:-C4 C5}; do
    for v in ${VARIANTS:-base prev}; do
      if [ "$v" = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$v.so; fi
      BHRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-host-path $EXTRA > $OUT/${cfg}_${v}_$round.json 2>$OUT/${cfg}_${v}_$round.err || { echo "$cfg $v failed"; tail -3 $OUT/${cfg}_${v}_$round.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$OUT/${cfg}_${v}_$round.json')); print('$cfg', '$v', $round, d['value'], d['kernel']['avg_ms'])"
    done
  done
done
