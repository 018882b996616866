#!/bin/bash
# Round-4 session AB: the slow batch mode vanished whenever timing events were recorded (HIP
# events with timing, or rocprofv3): which marker does it?
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for m in 0 4 8 12 16 31; do
    PRE_FRAMES=7 BHRT_BATCH_MARKERS=$m CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> /dev/null || { echo "probe failed"; exit 1; }
    echo "markers $m: $(grep -v 'num_threads 8' $OUT/bp.txt | sed 's/.*num_threads 0: //')"
  done
done
for m in 0 12; do
  BHRT_BATCH_MARKERS=$m timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_ab.json 2> /dev/null || { echo "bench failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_ab.json')); h=d['host_path']; print('bench markers $m', d['value'], 'batch', h['trace_rays_batch_mrays_s'], h['trace_rays_batch_after_frames_mrays_s'])"
done
echo all-done
