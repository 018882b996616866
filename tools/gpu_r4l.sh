#!/bin/bash
# Round-4 session L: GPU suite after the batch changes; trace_rays_batch default plan; default bench.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "== torch after libbhrt"
timeout -k 10 600 python3 tools/torch_after_lib.py || { echo "diag failed"; exit 1; }
for r in 1 2 3; do
  CHUNKS=4 timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2>/dev/null || { echo "probe failed"; exit 1; }
  echo "default plan $(head -1 $OUT/bp.txt | sed 's/.*num_threads 0: //')"
done
echo "== default bench" && timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
  || { echo "bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo all-done
