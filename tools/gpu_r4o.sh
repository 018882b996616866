#!/bin/bash
# Round-4 session O: trace_rays_batch inside bench.py (host-path leg) against the probe.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
BHRT_HOST_TIMING=1 timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_o.json 2> $OUT/bench_o.err || { echo "bench failed"; tail -20 $OUT/bench_o.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_o.json')); print('bench', d['value'], d['host_path'])"
grep "trace_rays_batch" $OUT/bench_o.err | tail -5
CHUNKS=x BHRT_HOST_TIMING=1 timeout -k 10 200 python3 tools/batch_probe.py 2> $OUT/bp_t.txt || exit 1
grep "trace_rays_batch" $OUT/bp_t.txt | tail -3
GPU_MAX_HW_QUEUES=8 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py || exit 1
echo all-done
