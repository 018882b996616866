#!/bin/bash
# Frames of CONFIGS rendered by the in-tree library and by ab/libbhrt_$REF.so, compared field by
# field (tools/diff_libs.py): shows whether a kernel change moves any output bit.
cd "$(dirname "$0")/.."
T=${TMPDIR:-/tmp}/bitexact; mkdir -p $T
for c in ${CONFIGS:-C3 C4 C5}; do
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_$REF.so timeout -k 10 300 python tools/diff_libs.py save $c $T/ref_$c.npz || exit 1
  timeout -k 10 300 python tools/diff_libs.py save $c $T/new_$c.npz || exit 1
  echo "== $c: in-tree vs $REF"
  python tools/diff_libs.py cmp $T/new_$c.npz $T/ref_$c.npz || exit 1
  rm -f $T/ref_$c.npz $T/new_$c.npz
done
