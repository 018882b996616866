#!/bin/bash
# Round-4 session R: why trace_rays_batch is slower inside bench.py's host-path leg than in the
# probe -- the GPU timeline of the leg's last batch call (kernels + copies).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_bench_r -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench_r.json 2> $OUT/bench_r.err || { echo "bench failed"; tail -20 $OUT/bench_r.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_r.json')); print('batch', d['host_path']['trace_rays_batch_mrays_s'])"
K=$(find $OUT/prof_bench_r -name "*kernel_trace.csv" | head -1); M=$(find $OUT/prof_bench_r -name "*memory_copy_trace.csv" | head -1)
python3 tools/batch_timeline.py $K $M --min-span 5 > $OUT/batch_timeline_r.txt || true
cat $OUT/batch_timeline_r.txt
python3 tools/batch_timeline.py $K $M --min-span 5 --call -2 | tail -1 || true
echo "== probe, same box"
CHUNKS=x timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof_probe_r -o run --output-format csv -- python3 tools/batch_probe.py > $OUT/probe_r.txt 2>&1 || { echo "probe failed"; exit 1; }
CHUNKS=x head -1 $OUT/probe_r.txt
K=$(find $OUT/prof_probe_r -name "*kernel_trace.csv" | head -1); M=$(find $OUT/prof_probe_r -name "*memory_copy_trace.csv" | head -1)
python3 tools/batch_timeline.py $K $M --min-span 5 | tail -1
echo all-done
