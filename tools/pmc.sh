#!/bin/bash
# rocprofv3 PMC passes over the trace kernel of bench.py (one counter group per pass,
# kernel-trace only; no sys/runtime traces with --pmc). $PMC_BENCH_ARGS: extra bench.py flags
# (e.g. "--fields display").
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf $OUT/p[0-9]*   # passes of an earlier run must not mix into this summary
mkdir -p $OUT
CFG=${CFG:-C2}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'k_trace<' --output-format csv \
      -d $OUT/p$i -o pass -- python bench.py --config $CFG --steps 1 --warmup 1 --streams 1 --no-cpu-baseline --no-host-path $PMC_BENCH_ARGS \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
