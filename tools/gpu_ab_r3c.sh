#!/bin/bash
# round-3 A/B: SGPR relief (kernel-argument loads at refill / store) on top of the v29 candidates
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_REHEARSE=1 AB_REF=rot AB_VARIANTS="cold" AB_CFGS="C2 C3 C4 C5" AB_ROUNDS=1 bash tools/gpu_r3.sh > gpurun_out/ab_cold.txt 2>&1 || { tail -20 gpurun_out/ab_cold.txt; exit 1; }
grep -c identical gpurun_out/ab_cold.txt
CFG=C3 VARIANTS="base28 rot cold coldc4" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C4 VARIANTS="base28 rotc4 cold coldc4" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C5 VARIANTS="base28 rotc4 cold coldc4" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C2 VARIANTS="base28 mo cold" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
