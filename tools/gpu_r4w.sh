#!/bin/bash
# Round-4 session W: bench.py's host-path leg (trace_rays_batch) with the process confined to
# one NUMA node's CPUs (taskset, before any GPU use) against unconfined.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for node in 0 1 free; do
    if [ $node = free ]; then pre=""; else pre="taskset -c $(cat /sys/devices/system/node/node$node/cpulist)"; fi
    timeout -k 10 400 $pre python bench.py --no-cpu-baseline > $OUT/bench_w.json 2> $OUT/bench_w.err || { echo "bench failed"; tail -20 $OUT/bench_w.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_w.json')); h=d['host_path']; print('node $node', d['value'], 'sync', h['mrays_s'], 'async', h['async_mrays_s'], 'rgba8', h['rgba8_mrays_s'], h['rgba8_async_mrays_s'], 'batch', h['trace_rays_batch_mrays_s'])"
  done
done
echo all-done
