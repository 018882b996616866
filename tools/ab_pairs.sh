#!/bin/bash
# Same-box interleaved A/B of (config, variant) pairs against the in-tree library:
#   PAIRS="C3:c3w3 C5:c5w5" ROUNDS=3 bash tools/ab_pairs.sh
# variant libraries: raytracing-engine-in-c_amd/ab/libbhrt_<variant>.so (make -C csrc OBJ=... OUT=...)
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab; mkdir -p $OUT
for round in $(seq ${ROUNDS:-3}); do
  for pair in $PAIRS; do
    cfg=${pair%%:*}; var=${pair##*:}
    for v in base $var; do
      if [ "$v" = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$v.so; fi
      BHRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-path $EXTRA > $OUT/${cfg}_${v}_$round.json 2>$OUT/${cfg}_${v}_$round.err || { echo "$cfg $v failed"; tail -3 $OUT/${cfg}_${v}_$round.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${cfg}_${v}_$round.json')); print('$cfg', '$v', $round, d['value'], d['kernel']['avg_ms'])"
    done
  done
done
