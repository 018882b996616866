#!/bin/bash
# Round-4 session G: bench.py --streams auto on every config (N = 1) and the C4 8-GPU-plan shard;
# the GPU timeline of one trace_rays_batch call (kernels + copies).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for ex in "--config C1" "--config C2" "--config C3" "--config C4" "--config C5" "--config C4 --plan-gpus 8 --shard 0"; do
  timeout -k 10 120 python bench.py $ex --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/g.json 2>/dev/null \
    || { echo "$ex failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/g.json')); print('$ex', d['value'], d['ms_per_step'], d['warmup'], d['kernel']['streams'], d['kernel']['streams_policy'])"
done
echo "== batch timeline"
CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_batch -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/batch_prof.txt 2> $OUT/batch_prof.err \
  || { echo "rocprof batch failed"; tail -20 $OUT/batch_prof.err; exit 1; }
cat $OUT/batch_prof.txt
python3 tools/batch_timeline.py $(find $OUT/prof_batch -name "*kernel_trace.csv" | head -1) $(find $OUT/prof_batch -name "*memory_copy_trace.csv" | head -1) > $OUT/batch_timeline.txt || true
cat $OUT/batch_timeline.txt
echo all-done
