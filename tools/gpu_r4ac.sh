#!/bin/bash
# Round-4 session AC: SALU of the Kerr RK4 iteration -- the disk test's 1e150 bound hoisted into
# an SGPR pair (in-tree "base") and the step size formed at the cache branch's join ("hc"),
# against the previous build ("base0"): bit-exactness, same-box rate, SALU/VALU counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
[ -n "$SKIP_BITEXACT" ] || { echo "== bit-exact vs base0" && REF=base0 CONFIGS="C2 C3 C4 C5" bash tools/ab_bitexact.sh || exit 1; }
echo "== bit-exact hc vs base0"
for c in C4 C2; do
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_hc.so timeout -k 10 300 python tools/diff_libs.py save $c /tmp/hc_$c.npz || exit 1
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_base0.so timeout -k 10 300 python tools/diff_libs.py save $c /tmp/b0_$c.npz || exit 1
  python tools/diff_libs.py cmp /tmp/hc_$c.npz /tmp/b0_$c.npz || exit 1
done
for c in C4 C2 C5; do
  echo "== ab $c" && CFG=$c VARIANTS="base0 base hc" ROUNDS=${ROUNDS:-3} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
done
echo "== pmc C4" && CFG=C4 VARIANTS="base0 base hc" CNT="SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc_ab.sh || exit 1
echo all-done
