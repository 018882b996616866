#!/bin/bash
# Round-4 session N: trace_rays_batch under torch's HIP runtime: hardware queues (4 / 8, as
# bench.py sets) and the runtime's copy-engine choice (GPU_BLIT_ENGINE_TYPE) for the D2H.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 GPU_BLIT_ENGINE_TYPE=1" "GPU_MAX_HW_QUEUES=8 GPU_BLIT_ENGINE_TYPE=2" "GPU_MAX_HW_QUEUES=8 BHRT_BATCH_WEIGHTS=1,1,1,1"; do
    env $v BHRT_HOST_TIMING=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> $OUT/bp_t.txt || { echo "probe failed"; tail -5 $OUT/bp_t.txt; exit 1; }
    echo "$v: $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
    sed -n 3p $OUT/bp_t.txt
  done
done
for v in 1 2; do
  GPU_MAX_HW_QUEUES=8 GPU_BLIT_ENGINE_TYPE=$v CHUNKS=x timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch_n$v -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
    || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
  echo "== timeline GPU_BLIT_ENGINE_TYPE=$v"
  python3 tools/batch_timeline.py $(find $OUT/prof_batch_n$v -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch_n$v -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline_n$v.txt || true
  grep -c "copyBuffer" $OUT/batch_timeline_n$v.txt || true
  tail -1 $OUT/batch_timeline_n$v.txt
done
echo all-done
