#!/bin/bash
# For base and each ablation: kernel time + iterations (bench.py) and SQ_INSTS_VALU per
# launch (rocprofv3 PMC on the hot k_trace instantiation) -> gpurun_out/ablation/*.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/ablation; mkdir -p $OUT
for v in base ${VARIANTS:-chain stageshift div clamp disk dist}; do
  if [ "$v" = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_x_$v.so; fi
  BHRT_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err || { echo "$v bench failed"; exit 1; }
  rm -rf $OUT/pmc_$v
  BHRT_LIB=$lib timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --kernel-include-regex 'k_trace<.*, false>' --output-format csv -d $OUT/pmc_$v -o pass -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_$v.log 2>&1 || { echo "$v pmc failed"; exit 1; }
  echo "$v done"
done
