#!/bin/bash
# Round-4 session AF: tiles claimed longest-first by the previous frame's steps (bench.py
# --claim-order prev-tiles, opt-in) against the default order.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for ex in "--config C4 --plan-gpus 8 --shard 0" "--config C4" "--config C2" "--config C5 --plan-gpus 8 --shard 0"; do
    for co in default prev-tiles; do
      timeout -k 10 150 python bench.py $ex --steps 30 --warmup 3 --no-cpu-baseline --no-host-path --claim-order $co > $OUT/af.json 2> $OUT/af.err || { echo "$ex $co failed"; tail -5 $OUT/af.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/af.json')); print('$ex', '$co', d['value'], d['ms_per_step'], d['kernel']['streams'], d['kernel'].get('claim_order'))"
    done
  done
done
echo all-done
