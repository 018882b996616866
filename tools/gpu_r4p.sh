#!/bin/bash
# Round-4 session P: trace_rays_batch after torch streams exist (bench.py's situation).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "PRE_STREAMS=0" "PRE_STREAMS=2" "PRE_STREAMS=4" "PRE_STREAMS=4 GPU_MAX_HW_QUEUES=8" "PRE_STREAMS=0 GPU_MAX_HW_QUEUES=8"; do
    env $v BHRT_HOST_TIMING=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
    echo "$v: $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
    sed -n 3p $OUT/bp_t.txt
  done
done
echo all-done
