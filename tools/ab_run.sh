#!/bin/bash
# One A/B session: GPU parity suite on the product build (+ $TEST_VARIANTS), interleaved bench
# rounds of $VARIANTS (tools/ab.sh), and the CPU-reference parity of the bench rows
# (class mismatches, max relative hit difference) for $CPU_VARIANTS.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/ab/pytest_base.log 2>&1 || { echo "pytest base failed"; tail -n 30 gpurun_out/ab/pytest_base.log; exit 1; }
echo "pytest base: $(tail -n 1 gpurun_out/ab/pytest_base.log)"
if [ -n "$TEST_VARIANTS" ]; then VARIANTS="$TEST_VARIANTS" bash tools/ab_tests.sh || exit 1; fi
VARIANTS="${VARIANTS:-base}" ROUNDS=${ROUNDS:-2} bash tools/ab.sh || exit 1
for v in ${CPU_VARIANTS:-base}; do
  if [ $v = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$v.so; fi
  BHRT_LIB=$lib timeout -k 10 300 python bench.py --config ${CFG:-C2} --steps 3 --warmup 1 --no-host-path > gpurun_out/ab/cpu_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/cpu_$v.json')); print('cpu-parity $v', d['value'], d['class_mismatch'], d['max_rel_dhit'])"
done
