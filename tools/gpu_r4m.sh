#!/bin/bash
# Round-4 session M: trace_rays_batch under torch's bundled HIP runtime (bhrt.lib imports torch
# first) against /opt/rocm's (BHRT_PY_NO_TORCH=1): per-call breakdown and the GPU timeline.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for nt in 0 1; do
    for w in "1,3,3,3,1" "1,1,1,1"; do
      BHRT_PY_NO_TORCH=$nt BHRT_BATCH_WEIGHTS=$w BHRT_HOST_TIMING=1 CHUNKS=4 timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; exit 1; }
      echo "no_torch=$nt w=$w $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
      sed -n 3,4p $OUT/bp_t.txt
    done
  done
done
for nt in 0 1; do
  BHRT_PY_NO_TORCH=$nt CHUNKS=4 BHRT_BATCH_WEIGHTS="1,3,3,3,1" timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch_m$nt -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
    || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
  echo "== timeline no_torch=$nt"
  python3 tools/batch_timeline.py $(find $OUT/prof_batch_m$nt -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch_m$nt -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline_m$nt.txt || true
  cat $OUT/batch_timeline_m$nt.txt
done
echo all-done
