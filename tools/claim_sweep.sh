#!/bin/bash
# Same-box A/B of the ray-queue / claim policy (BHRT_QUEUES, BHRT_QUEUE_STRIDE, BHRT_CLAIM_DIV,
# BHRT_CLAIM_MIN): every config x setting "Q:stride:div:min", interleaved over
# $ROUNDS rounds; one line per run.
cd "$(dirname "$0")/.."
OUT=gpurun_out/claim; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-C3 C4 C5 C2}; do
    for s in ${SETTINGS:-1:32:0:64 16:32:0:64}; do
      IFS=: read q st d m <<< "$s"
      tag=$c.$q.$st.$d.$m.$r
      BHRT_QUEUES=$q BHRT_QUEUE_STRIDE=$st BHRT_CLAIM_DIV=$d BHRT_CLAIM_MIN=$m timeout -k 10 300 \
          python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-path \
          > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$r $c Q=$q stride=$st div=$d min=$m', d['value'], 'kern', d['kernel']['avg_ms'], 'frac', d['roofline']['frac'])"
    done
  done
done
