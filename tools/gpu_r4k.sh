#!/bin/bash
# Round-4 session K: shared-origin batches upload directions only; chunk plans again; timeline.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== torch after libbhrt"
timeout -k 10 600 python3 tools/torch_after_lib.py || { echo "diag failed"; exit 1; }
echo "== batch tests"
for w in "" "1,3,3,1"; do
  BHRT_BATCH_WEIGHTS="$w" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batch or shared_origin or rays_vs" > $OUT/pytest_batch_k.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_batch_k.log; exit 1; }
  tail -1 $OUT/pytest_batch_k.log
done
for r in 1 2 3; do
  for w in "" "1,3,3,1" "2,3,3,1" "1,3,3,2" "1,2,2,1" "1,3,3,3,1"; do
    BHRT_BATCH_WEIGHTS="$w" CHUNKS=4 timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2>/dev/null || { echo "probe failed"; exit 1; }
    echo "w=[$w] $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
  done
done
echo "== timeline 1,3,3,1"
BHRT_BATCH_WEIGHTS="1,3,3,1" CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch_k -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
  || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
cat $OUT/batch_prof.txt
python3 tools/batch_timeline.py $(find $OUT/prof_batch_k -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch_k -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline_k.txt || true
cat $OUT/batch_timeline_k.txt
echo all-done
