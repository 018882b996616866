#!/bin/bash
# Round-4 session B: GPU parity suite -> same-box A/B of host/launch knobs on C4 (whole frame and
# one shard of the 8-GPU plan) and C5 -> rocprofv3 of a C4 plan shard, serial frames -> the
# trace_rays_batch probe -> C4 plan shards. A failing test does not stop the session (rc 1);
# a crash, abort or time limit does.
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
KNOBS=${KNOBS:-"base base:BHRT_FUSE_COLOUR=0 base:BHRT_SKIP_REDO=0 base:BHRT_CLAIM_DIV=0 base:BHRT_CLAIM_DIV=4"}
if [ -z "$SKIP_AB" ]; then
  echo "== ab C4" && CFG=C4 VARIANTS="$KNOBS" ROUNDS=${AB_ROUNDS:-3} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
  echo "== ab C4 plan-8 shard 0" && CFG=C4 VARIANTS="$KNOBS" ROUNDS=${AB_ROUNDS:-3} EXTRA="--no-host-path --plan-gpus 8 --shard 0" bash tools/ab.sh || exit 1
  echo "== ab C5" && CFG=C5 VARIANTS="base base:BHRT_CLAIM_DIV=0 base:BHRT_CLAIM_DIV=4 base:BHRT_SKIP_REDO=0" ROUNDS=${AB_ROUNDS:-3} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
fi
for v in ${TRACE_VARIANTS-p8s1 p8s2}; do
  case $v in
    p8s1) args="--plan-gpus 8 --shard 0 --streams 1";;
    p8s2) args="--plan-gpus 8 --shard 0";;
  esac
  echo "== rocprof C4 $v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C4_$v -o run --output-format csv -- python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path $args > $OUT/bench_prof_C4_$v.json 2> $OUT/prof_C4_$v.err \
    || { echo "rocprof C4 $v failed"; tail -20 $OUT/prof_C4_$v.err; exit 1; }
  python tools/frame_timeline.py $(find $OUT/prof_C4_$v -name "*kernel_trace.csv" | head -1) --skip 3 > $OUT/timeline_C4_$v.txt || true
  cat $OUT/timeline_C4_$v.txt
done
if [ -z "$SKIP_BATCH" ]; then
  echo "== batch probe"
  CHUNKS="4 3 6" BHRT_HOST_TIMING=1 timeout -k 10 300 python tools/batch_probe.py > $OUT/batch_probe.txt 2> $OUT/batch_probe.err \
    || { echo "batch probe failed"; tail -20 $OUT/batch_probe.err; exit 1; }
  cat $OUT/batch_probe.txt
fi
if [ -z "$SKIP_PLAN" ]; then
  echo "== plan shards"
  CONFIGS="${PLAN_CFGS:-C4}" bash tools/plan_shards.sh > $OUT/plan_shards.jsonl 2> $OUT/plan_shards.err \
    || { echo "plan shards failed"; tail -20 $OUT/plan_shards.err; exit 1; }
  python tools/plan_summary.py $OUT/plan_shards.jsonl --out $OUT/plan_summary.txt
fi
if [ -n "${PMC_CFGS-C4 C5}" ]; then
  echo "== pmc" && CONFIGS="${PMC_CFGS-C4 C5}" bash tools/pmc_all.sh || exit 1
fi
echo all-done
