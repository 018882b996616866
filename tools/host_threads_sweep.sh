#!/bin/bash
# Host-path rate vs the host un-permute thread count (BHRT_HOST_THREADS), C2, 2 rounds.
cd "$(dirname "$0")/.."
OUT=gpurun_out/hostthreads; mkdir -p $OUT
for round in 1 2; do
  for t in ${THREADS:-4 8 12 16}; do
    BHRT_HOST_THREADS=$t timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/t${t}_$round.json 2> $OUT/t${t}_$round.err || { echo "threads $t failed"; tail -3 $OUT/t${t}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/t${t}_$round.json')); h=d['host_path']; print('threads', $t, $round, 'resident', d['value'], 'sync', h['mrays_s'], 'async', h['async_mrays_s'], 'batch', h.get('trace_rays_batch_mrays_s'))"
  done
done
