#!/bin/bash
# Round-4 session AE: Kerr paths' trip guard without the large-argument flag (nothing in their
# loop can raise it; a ray flagged at refill runs the trip out and is handed over, as before).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in C4 C5; do
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_nh.so timeout -k 10 300 python tools/diff_libs.py save $c /tmp/nh_$c.npz || exit 1
  timeout -k 10 300 python tools/diff_libs.py save $c /tmp/b_$c.npz || exit 1
  echo "== $c nh vs base"; python tools/diff_libs.py cmp /tmp/nh_$c.npz /tmp/b_$c.npz | grep -v identical || true
done
for c in C4 C5; do
  echo "== ab $c" && CFG=$c VARIANTS="base nh" ROUNDS=4 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
done
echo "== pmc C4" && CFG=C4 VARIANTS="base nh" CNT="SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc_ab.sh || exit 1
echo all-done
