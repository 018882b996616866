#!/bin/bash
# PMC passes (tools/pmc.sh) over the hot trace kernel of every config in $CONFIGS; each
# config's summary lands in gpurun_out/pmc_<CFG>$PMC_SUFFIX.json (copy into profiles/ to commit);
# $PMC_BENCH_ARGS goes to every profiled bench.py (tools/pmc.sh).
cd "$(dirname "$0")/.."
# PMC_EXTRA=1 adds two passes that split the waiting: scalar-memory, LDS and
# vector-memory instruction counts and their issue/wait cycles
PASSES=("SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES"
        "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
        "GRBM_GUI_ACTIVE FETCH_SIZE" "WRITE_SIZE")
if [ -n "$PMC_EXTRA" ]; then
  PASSES+=("SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES"
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES")
fi
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  CFG=$c bash tools/pmc.sh "${PASSES[@]}" > gpurun_out/pmc_$c$PMC_SUFFIX.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c$PMC_SUFFIX.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc $c gpurun_out/pmc_$c$PMC_SUFFIX.json > /dev/null || exit 1
  mkdir -p gpurun_out/pmc_raw_$c$PMC_SUFFIX && cp -r gpurun_out/pmc/p[0-9]* gpurun_out/pmc_raw_$c$PMC_SUFFIX/
  echo "pmc $c ok"
done
