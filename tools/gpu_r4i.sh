#!/bin/bash
# Round-4 session I: trace_rays_batch chunk plans (BHRT_BATCH_WEIGHTS) on C2's 2 M camera rays.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== batch tests with a weighted plan"
BHRT_BATCH_WEIGHTS="1,5,5,4,1" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batch or shared_origin" > $OUT/pytest_batch_w.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/pytest_batch_w.log; exit 1; }
tail -1 $OUT/pytest_batch_w.log
for r in 1 2; do
  for w in "" "1,5,5,4,1" "1,3,3,1" "1,6,6,3" "2,5,5,3,1" "1,7,7,1" "1,4,4,4,4,4,4,1" "1,2,2,2,1"; do
    BHRT_BATCH_WEIGHTS="$w" CHUNKS=4 timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2>/dev/null || { echo "probe failed"; exit 1; }
    echo "w=[$w] $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
  done
done
echo all-done
