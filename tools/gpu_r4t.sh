#!/bin/bash
# Round-4 session T: does a host-frame leg before the batch calls slow them (bench.py's order)?
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "PRE_FRAMES=0" "PRE_FRAMES=1" "PRE_FRAMES=8" "PRE_FRAMES=8 PRE_STREAMS=2"; do
    env $v BHRT_HOST_TIMING=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
    echo "$v: $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
    grep "trace_rays_batch n=" $OUT/bp_t.txt | sed -n 3p
  done
done
echo all-done
