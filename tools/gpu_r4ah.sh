#!/bin/bash
# Round-4 session AH: iterations per trip of the persistent loop re-swept on the current kernels
# (RK4 4/5/6/8 on C2 and C4, RKF45 1/2/3 on C3 and C5).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
echo "== ab C2" && CFG=C2 VARIANTS="base u4 u5 u8" ROUNDS=3 EXTRA="--no-host-path --steps 10" bash tools/ab.sh || exit 1
echo "== ab C4" && CFG=C4 VARIANTS="base u4 u5 u8" ROUNDS=3 EXTRA="--no-host-path --steps 20" bash tools/ab.sh || exit 1
echo "== ab C3" && CFG=C3 VARIANTS="base r1 r3" ROUNDS=3 EXTRA="--no-host-path --steps 30" bash tools/ab.sh || exit 1
echo "== ab C5" && CFG=C5 VARIANTS="base r1 r3" ROUNDS=3 EXTRA="--no-host-path --steps 20" bash tools/ab.sh || exit 1
echo all-done
