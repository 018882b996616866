#!/bin/bash
# Same-box A/B of kernel variants (ab/libbhrt_<v>.so) against ab/libbhrt_$AB_REF.so: each
# variant's full frames are first compared bit for bit with the reference build
# (tools/ab_bitexact.sh over $AB_BITEXACT_CFGS), then bench.py runs interleaved over $AB_CFGS.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$AB_VARIANTS" ]; then
  for v in $AB_VARIANTS; do
    echo "== bitexact $v vs $AB_REF"
    cp raytracing-engine-in-c_amd/libbhrt.so /tmp/libbhrt_intree.so
    cp raytracing-engine-in-c_amd/ab/libbhrt_$v.so raytracing-engine-in-c_amd/libbhrt.so
    REF=$AB_REF CONFIGS="${AB_BITEXACT_CFGS:-C1 C2 C3 C4 C5}" bash tools/ab_bitexact.sh > $OUT/bitexact_$v.txt 2>&1
    rc=$?
    cp /tmp/libbhrt_intree.so raytracing-engine-in-c_amd/libbhrt.so
    cat $OUT/bitexact_$v.txt
    [ $rc -eq 0 ] || { echo "bitexact failed"; exit 1; }
  done
  for c in ${AB_CFGS:-C2 C3}; do
    echo "== ab $c"
    CFG=$c VARIANTS="$AB_REF $AB_VARIANTS" ROUNDS=${AB_ROUNDS:-2} EXTRA="--no-host-path" bash tools/ab.sh || exit 1
  done
fi
echo ab-done
