#!/bin/bash
# Round-4 session Q: libbhrt's own streams made so that they get queues of their own
# (BHRT_STREAM_QUEUE 0/1/2) -- trace_rays_batch after torch streams exist, and inside bench.py.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for q in 0 1 2; do
    for v in "PRE_STREAMS=0" "PRE_STREAMS=2" "PRE_STREAMS=3 GPU_MAX_HW_QUEUES=8"; do
      env $v BHRT_STREAM_QUEUE=$q CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
      echo "queue=$q $v: $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
    done
  done
done
for q in 0 1 2; do
  BHRT_STREAM_QUEUE=$q timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_q.json 2> $OUT/bench_q.err || { echo "bench failed"; tail -20 $OUT/bench_q.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_q.json')); h=d['host_path']; print('bench queue=$q', d['value'], 'sync', h['mrays_s'], 'async', h['async_mrays_s'], 'rgba8', h['rgba8_mrays_s'], h['rgba8_async_mrays_s'], 'batch', h['trace_rays_batch_mrays_s'])"
done
echo all-done
