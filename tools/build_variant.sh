#!/bin/bash
# Build a kernel variant from the working tree with one text substitution in geodesic.hip:
# tools/build_variant.sh NAME 'python-expression-on-s' -> raytracing-engine-in-c_amd/ab/libbhrt_NAME.so
# e.g. tools/build_variant.sh w5 "s.replace('SPIN0) ? 4', 'SPIN0) ? 5')"
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXPR=$2
T=$(mktemp -d)
mkdir -p "$T/raytracing-engine-in-c_amd" raytracing-engine-in-c_amd/ab
cp -r raytracing-engine-in-c_amd/csrc "$T/raytracing-engine-in-c_amd/"
cp -r include "$T/"
rm -f "$T"/raytracing-engine-in-c_amd/csrc/*.o
python3 - "$T/raytracing-engine-in-c_amd/csrc/geodesic.hip" "$EXPR" <<'PY'
import sys
p, e = sys.argv[1], sys.argv[2]
s = open(p).read()
t = eval(e)
assert t != s, "substitution changed nothing"
open(p, "w").write(t)
PY
make -s -C "$T/raytracing-engine-in-c_amd/csrc" OUT="$PWD/raytracing-engine-in-c_amd/ab/libbhrt_$NAME.so" >/dev/null
rm -rf "$T"
echo "built ab/libbhrt_$NAME.so"
