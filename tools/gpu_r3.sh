#!/bin/bash
# Round-3 GPU session: GPU parity suite -> default bench (N = 1) -> the N-rank bench path
# rehearsed on one GPU (bench.py launches its own ranks; BHRT_BENCH_SHARE_DEVICE maps them all
# to GPU 0 over gloo, since RCCL refuses two ranks on one device). Every GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
if [ -z "$SKIP_BENCH" ]; then
  echo "== bench" && timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
for n in ${REHEARSE_N:-2 4}; do
  for c in ${REHEARSE_CFGS:-C2 C5}; do
    echo "== rehearsal --gpus $n --config $c"
    BHRT_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus $n --config $c --steps 4 --warmup 1 \
      > $OUT/rehearse_${n}_$c.json 2> $OUT/rehearse_${n}_$c.err \
      || { echo "rehearsal failed"; tail -30 $OUT/rehearse_${n}_$c.err; exit 1; }
    cat $OUT/rehearse_${n}_$c.json
  done
done
echo done
