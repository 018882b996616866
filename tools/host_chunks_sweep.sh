#!/bin/bash
# Host-buffer frame rate (bench.py host_path: sync, async, trace_ray latency) per chunk count,
# pinned staging (default) vs DMA into the registered caller arrays (BHRT_HOST_REGISTER=1).
cd "$(dirname "$0")/.."
OUT=gpurun_out/hostk; mkdir -p $OUT
for cfg in ${CONFIGS:-C2}; do
  for k in ${CHUNKS:-1 2 3 4 8}; do
    for stg in "" 1; do
      BHRT_HOST_CHUNKS=$k BHRT_HOST_REGISTER=$stg timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$cfg.$k.$stg.json 2> $OUT/$cfg.$k.$stg.err || { echo "$cfg $k failed"; tail -5 $OUT/$cfg.$k.$stg.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/$cfg.$k.$stg.json'))['host_path']; print('$cfg chunks=$k register=${stg:-0}', d)"
    done
  done
done
