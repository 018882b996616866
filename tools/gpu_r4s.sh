#!/bin/bash
# Round-4 session S: trace_rays_batch inside bench.py under different bench settings.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in "--steps 3 --warmup 1" "" "--steps 3 --warmup 1 --streams 2" "--streams 2" "--streams 1"; do
  BHRT_HOST_TIMING=1 timeout -k 10 400 python bench.py --no-cpu-baseline $v > $OUT/bench_s.json 2> $OUT/bench_s.err || { echo "bench failed"; tail -20 $OUT/bench_s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_s.json')); h=d['host_path']; print('[$v]', d['value'], d['kernel']['streams'], 'batch', h['trace_rays_batch_mrays_s'])"
  grep "trace_rays_batch n=" $OUT/bench_s.err | tail -2
done
echo all-done
