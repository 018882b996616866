SKIP_TESTS=1 SKIP_BENCH=1 SKIP_REHEARSE=1 AB_REF=base28 AB_VARIANTS="mo" AB_CFGS="C2 C4" AB_ROUNDS=1 bash tools/gpu_r3.sh > gpurun_out/ab_mo.txt 2>&1 || { tail -20 gpurun_out/ab_mo.txt; exit 1; }
grep -c identical gpurun_out/ab_mo.txt
timeout -k 10 300 python tools/full_frame_parity.py --configs C4 C5 --out gpurun_out/ffp_rot.json > gpurun_out/ffp_rot.txt 2>&1 || { tail -5 gpurun_out/ffp_rot.txt; exit 1; }
tail -1 gpurun_out/ffp_rot.txt
CFG=C3 VARIANTS="base28 mou3" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C4 VARIANTS="base28 mo rot rotc4" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C5 VARIANTS="base28 mo rot rotc4" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C2 VARIANTS="base28 mo" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
CFG=C3 VARIANTS="base28 mo mou1 mou3" ROUNDS=2 EXTRA="--no-host-path" bash tools/ab.sh || exit 1
