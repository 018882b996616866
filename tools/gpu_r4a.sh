#!/bin/bash
# Round-4 session A: GPU parity suite (every ray of C1-C4 and C5 shard 0) -> same-box A/B of
# kernel variants -> the 8-GPU plans' shards timed on one GPU -> rocprofv3 kernel traces of C4
# (serial frames, the bench's two streams, an 8-GPU-plan shard) -> trace_rays_batch probe.
# A failing test does not stop the session (rc 1); a crash, abort or time limit does.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
  rc=$?
  tail -1 $OUT/pytest_gpu.log
  grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
  [ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; tail -30 $OUT/pytest_gpu.log; exit 1; }
fi
for v in $BITEXACT_VARIANTS; do  # every field of full frames: in-tree library vs ab/libbhrt_$v.so
  echo "== bitexact in-tree vs $v"
  REF=$v CONFIGS="${BITEXACT_CFGS:-C2 C3 C4 C5}" bash tools/ab_bitexact.sh > $OUT/bitexact_$v.txt 2>&1 \
    || { echo "bitexact $v failed"; tail -20 $OUT/bitexact_$v.txt; exit 1; }
  cat $OUT/bitexact_$v.txt
done
if [ -n "$AB_VARIANTS" ]; then
  for c in ${AB_CFGS:-C4 C5}; do
    echo "== ab $c"
    CFG=$c VARIANTS="$AB_VARIANTS" ROUNDS=${AB_ROUNDS:-3} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
  done
fi
if [ -z "$SKIP_PLAN" ]; then
  echo "== plan shards"
  CONFIGS="${PLAN_CFGS:-C2 C4 C5}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
    || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
  python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
fi
for v in ${TRACE_VARIANTS-s1 s2 p8}; do
  case $v in
    s1) args="--streams 1";;
    s2) args="";;
    p8) args="--plan-gpus 8 --shard 0";;
  esac
  echo "== rocprof C4 $v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C4_$v -o run --output-format csv -- python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path $args > $OUT/bench_prof_C4_$v.json 2> $OUT/prof_C4_$v.err \
    || { echo "rocprof C4 $v failed"; tail -20 $OUT/prof_C4_$v.err; exit 1; }
  python tools/frame_timeline.py $(find $OUT/prof_C4_$v -name "*kernel_trace.csv" | head -1) --skip 3 > $OUT/timeline_C4_$v.txt || true
  cat $OUT/timeline_C4_$v.txt
done
if [ -z "$SKIP_BATCH" ]; then
  echo "== batch probe"
  BHRT_HOST_TIMING=1 timeout -k 10 300 python tools/batch_probe.py > $OUT/batch_probe.txt 2> $OUT/batch_probe.err \
    || { echo "batch probe failed"; tail -20 $OUT/batch_probe.err; exit 1; }
  cat $OUT/batch_probe.txt
fi
echo all-done
