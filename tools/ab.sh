#!/bin/bash
# A/B of libbhrt build variants on the bench workload (interleaved rounds). A variant is
# NAME (raytracing-engine-in-c_amd/ab/libbhrt_NAME.so; "base" = the in-tree library) or
# NAME:VAR=VALUE[,VAR=VALUE...] (the same library with environment variables set, e.g.
# fc:BHRT_FUSE_COLOUR=0).
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab; mkdir -p $OUT
CFG=${CFG:-C2}
VARIANTS=${VARIANTS:-"base"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    name=${v%%:*}; envset=""; [ "$name" != "$v" ] && envset=${v#*:} && envset=${envset//,/ }
    if [ "$name" = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$name.so; fi
    tag=$(echo "$v" | tr ':=' '__')
    env $envset BHRT_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline $EXTRA > $OUT/${CFG}_${tag}_$round.json 2>$OUT/${CFG}_${tag}_$round.err || { echo "$v failed"; tail -3 $OUT/${CFG}_${tag}_$round.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${CFG}_${tag}_$round.json')); print('$CFG', '$v', $round, d['value'], d['kernel']['avg_ms'])"
  done
done
