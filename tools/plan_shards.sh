#!/bin/bash
# Every rank's work of the 8-GPU runs, timed on one GPU: for each config
# the N = 1 line, then shard k of the N-GPU plan (bench.py --plan-gpus N --shard k) for every k.
# tools/plan_summary.py turns the lines into load balance and predicted scaling efficiency.
#   STEPS=20 N=8 CONFIGS="C2 C4 C5" tools/plan_shards.sh > gpurun_out/plan_shards.jsonl
# BENCH_ARGS adds bench.py options to every run (e.g. "--streams 4").
set -e -o pipefail
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-3}
N=${N:-8}
for cfg in ${CONFIGS:-C2 C4 C5}; do
    timeout -k 10 120 python3 bench.py --config "$cfg" --steps "$STEPS" --warmup "$WARMUP" \
        --no-cpu-baseline --no-host-path $BENCH_ARGS
    for k in $(seq 0 $((N - 1))); do
        timeout -k 10 120 python3 bench.py --config "$cfg" --plan-gpus "$N" --shard "$k" \
            --steps "$STEPS" --warmup "$WARMUP" --no-cpu-baseline --no-host-path $BENCH_ARGS
    done
done
