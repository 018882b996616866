#!/bin/bash
# Round-4 session AD: the AC A/B again on another box, more rounds, with SALU/VALU counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in C4 C2 C5; do
  echo "== ab $c" && CFG=$c VARIANTS="base0 base hc" ROUNDS=4 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
done
for c in C4 C2; do
  echo "== pmc $c" && CFG=$c VARIANTS="base0 base hc" CNT="SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc_ab.sh || exit 1
done
echo all-done
