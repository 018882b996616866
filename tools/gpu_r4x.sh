#!/bin/bash
# Round-4 session X: which of bench.py's legs before the batch calls puts a process in the
# slow trace_rays_batch mode (143 instead of 200 Mrays/s)? Fresh process per case, twice.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "PRE_FRAMES=0" "PRE_FRAMES=7" "PRE_ASYNC=9" "PRE_DEVICE=12" "PRE_DEVICE=12 PRE_FRAMES=7 PRE_ASYNC=9"; do
    env $v BHRT_HOST_TIMING=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
    echo "$v: $(grep -v 'num_threads 8' $OUT/bp.txt | sed 's/.*num_threads 0: //')"
  done
done
echo all-done
