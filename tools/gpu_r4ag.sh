#!/bin/bash
# Round-4 session AG: the claim/refill knobs again on the C4 8-GPU-plan shard, now with four
# frames in flight (--streams auto).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=C4 VARIANTS="base base:BHRT_REFILL=32 base:BHRT_REFILL=16 base:BHRT_CLAIM_DIV=2 base:BHRT_CLAIM_DIV=0 base:BHRT_QUEUES=32 base:BHRT_TRACE_BLOCK=128" ROUNDS=3 EXTRA="--no-host-path --plan-gpus 8 --shard 0 --steps 30" bash tools/ab.sh || exit 1
echo all-done
