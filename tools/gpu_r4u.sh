#!/bin/bash
# Round-4 session U: the bimodal trace_rays_batch rate (203 or 144 Mrays/s per process): CPU /
# NUMA placement of the probe process, and the rate, over several fresh processes.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3 4 5 6; do
  WHERE=1 PRE_FRAMES=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> /dev/null || { echo "probe failed"; exit 1; }
  cat $OUT/bp.txt | grep -v "num_threads 8" | tr '\n' ' '; echo
done
echo all-done
