#!/bin/bash
# round-3 A/B: init-table loads through the kernel-argument pointer (ld) and occupancy variants
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_REHEARSE=1 AB_REF=cold AB_VARIANTS="ld" AB_CFGS="C2 C3 C4 C5" AB_ROUNDS=1 bash tools/gpu_r3.sh > gpurun_out/ab_ld.txt 2>&1 || { tail -20 gpurun_out/ab_ld.txt; exit 1; }
grep -c identical gpurun_out/ab_ld.txt
CFG=C3 VARIANTS="cold ld c3w3" ROUNDS=3 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C4 VARIANTS="cold ld c4w5" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C5 VARIANTS="cold ld c5w5" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C2 VARIANTS="cold ld" ROUNDS=3 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
