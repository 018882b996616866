#!/bin/bash
# Round-4 session AA: does earlier pinned-memory use put a process in the slow batch mode?
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "PRE_FRAMES=0" "PRE_FRAMES=7" "PRE_PIN=600" "PRE_PIN=600 PRE_PIN_KEEP=1" "PRE_PAGEABLE=4"; do
    env $v BHRT_HOST_TIMING=2 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
    echo "$v: $(grep -v 'num_threads 8' $OUT/bp.txt | sed 's/.*num_threads 0: //')"
    grep -A5 "trace_rays_batch n=" $OUT/bp_t.txt | sed -n 14,15p
  done
done
echo all-done
