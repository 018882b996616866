#!/bin/bash
# Round-4 session J: more trace_rays_batch chunk plans, and the GPU timeline of the best one.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "W=1,3,3,1" "W=1,2,2,1" "W=1,3,3,2" "W=1,2,3,3,1" "W=1,4,4,1" "W=1,3,3,1 S=3" "W=2,3,3,1" "W=1,3,3,3,1"; do
    w=$(echo $v | sed 's/.*W=\([0-9,]*\).*/\1/'); st=2; case "$v" in *S=3*) st=3;; esac
    BHRT_BATCH_STREAMS=$st BHRT_BATCH_WEIGHTS="$w" CHUNKS=4 timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2>/dev/null || { echo "probe failed"; exit 1; }
    echo "$v $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
  done
done
echo "== timeline 1,3,3,1"
BHRT_BATCH_WEIGHTS="1,3,3,1" CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch_j -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
  || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
cat $OUT/batch_prof.txt
python3 tools/batch_timeline.py $(find $OUT/prof_batch_j -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch_j -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline_j.txt || true
cat $OUT/batch_timeline_j.txt
echo all-done
