#!/bin/bash
# gpu_check (smoke, parity suite, bench, kernel trace) then PMC passes for the roofline traffic.
cd "$(dirname "$0")/.."
bash tools/gpu_check.sh || exit 1
bash tools/pmc.sh "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE FETCH_SIZE" "WRITE_SIZE" > gpurun_out/pmc.log 2>&1 && echo pmc ok
