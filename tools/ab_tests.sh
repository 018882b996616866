#!/bin/bash
# GPU parity suite against A/B build variants.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-ctr fs}; do
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_$v.so timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/ab/pytest_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
