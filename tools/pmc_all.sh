#!/bin/bash
# PMC passes (tools/pmc.sh) over the hot trace kernel of every config in $CONFIGS; each
# config's summary lands in gpurun_out/pmc_<CFG>.json (copy into profiles/ to commit).
cd "$(dirname "$0")/.."
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  CFG=$c bash tools/pmc.sh "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES" \
      "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
      "GRBM_GUI_ACTIVE FETCH_SIZE" "WRITE_SIZE" > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc $c gpurun_out/pmc_$c.json > /dev/null || exit 1
  mkdir -p gpurun_out/pmc_raw_$c && cp -r gpurun_out/pmc/p[0-9]* gpurun_out/pmc_raw_$c/
  echo "pmc $c ok"
done
