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
[ -n "$SKIP_REHEARSE" ] || for n in ${REHEARSE_N:-2 4}; do
  for c in ${REHEARSE_CFGS:-C2 C5}; do
    echo "== rehearsal --gpus $n --config $c"
    BHRT_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus $n --config $c --steps 4 --warmup 1 \
      > $OUT/rehearse_${n}_$c.json 2> $OUT/rehearse_${n}_$c.err \
      || { echo "rehearsal failed"; tail -30 $OUT/rehearse_${n}_$c.err; exit 1; }
    cat $OUT/rehearse_${n}_$c.json
  done
done
echo done
# optional same-box A/B of kernel variants (ab/libbhrt_<v>.so) against REF, with the full-frame
# bit-exact comparison first (tools/ab_bitexact.sh)
if [ -n "$AB_VARIANTS" ]; then
  for v in $AB_VARIANTS; do
    echo "== bitexact $v vs $AB_REF"
    cp raytracing-engine-in-c_amd/libbhrt.so /tmp/libbhrt_intree.so
    cp raytracing-engine-in-c_amd/ab/libbhrt_$v.so raytracing-engine-in-c_amd/libbhrt.so
    REF=$AB_REF CONFIGS="${AB_CFGS:-C2 C3 C4 C5}" bash tools/ab_bitexact.sh > $OUT/bitexact_$v.txt 2>&1
    rc=$?
    cp /tmp/libbhrt_intree.so raytracing-engine-in-c_amd/libbhrt.so
    cat $OUT/bitexact_$v.txt
    [ $rc -eq 0 ] || { echo "bitexact failed"; exit 1; }
  done
  for c in ${AB_CFGS:-C2 C3 C4 C5}; do
    echo "== ab $c"
    CFG=$c VARIANTS="$AB_REF $AB_VARIANTS" ROUNDS=${AB_ROUNDS:-2} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
  done
fi
echo all-done
