#!/bin/bash
# Build libbhrt.so of git revision REV into raytracing-engine-in-c_amd/ab/libbhrt_NAME.so (A/B
# against an earlier kernel on the same box). Usage: tools/build_rev.sh REV NAME [DEFS]
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2; DEFS=${3:-}
T=$(mktemp -d)
git archive "$REV" raytracing-engine-in-c_amd/csrc include | tar -x -C "$T"
make -s -C "$T/raytracing-engine-in-c_amd/csrc" OUT="$PWD/raytracing-engine-in-c_amd/ab/libbhrt_$NAME.so" DEFS="$DEFS" >/dev/null
rm -rf "$T"
echo "built ab/libbhrt_$NAME.so from $REV"
