#!/bin/bash
# Round-4 session H: ray arrays with one shared origin set up in the trace kernel, the control
# region reset by a DMA copy. GPU suite, then trace_rays_batch (shared origin on/off, copy/fill
# reset), its timeline, and the copy/fill reset A/B on frames.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
echo "== batch probe"
for v in "BHRT_SHARED_ORIGIN=1 BHRT_CTL_COPY=1" "BHRT_SHARED_ORIGIN=0 BHRT_CTL_COPY=1" "BHRT_SHARED_ORIGIN=1 BHRT_CTL_COPY=0" "BHRT_SHARED_ORIGIN=0 BHRT_CTL_COPY=0"; do
  echo "-- $v"
  env $v CHUNKS="4 3 6" BHRT_HOST_TIMING=1 timeout -k 10 200 python3 tools/batch_probe.py 2> $OUT/batch_probe_timing.txt || { echo "batch probe failed"; exit 1; }
  grep "K=4" $OUT/batch_probe_timing.txt | tail -2
done
echo "== batch timeline"
CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch_h -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
  || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
cat $OUT/batch_prof.txt
python3 tools/batch_timeline.py $(find $OUT/prof_batch_h -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch_h -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline_h.txt || true
cat $OUT/batch_timeline_h.txt
echo "== ctl reset A/B on frames"
for r in 1 2; do
  for ex in "--config C4 --plan-gpus 8 --shard 0" "--config C3" "--config C4" "--config C2"; do
    for cc in 1 0; do
      BHRT_CTL_COPY=$cc timeout -k 10 120 python bench.py $ex --steps 30 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/h.json 2>/dev/null \
        || { echo "$ex failed"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/h.json')); print('$ex ctl_copy=$cc', d['value'], d['ms_per_step'], d['kernel']['streams'])"
    done
  done
done
echo all-done
