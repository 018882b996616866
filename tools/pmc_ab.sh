#!/bin/bash
# PMC counters (one pass) of the hot k_trace launch for each A/B variant: ab/pmc_<v>.csv
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/ab; mkdir -p $OUT
CNT=${CNT:-"SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"}
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then lib=raytracing-engine-in-c_amd/libbhrt.so; else lib=raytracing-engine-in-c_amd/ab/libbhrt_$v.so; fi
  rm -rf $OUT/pmc_$v
  BHRT_LIB=$lib timeout -k 10 200 rocprofv3 --pmc $CNT --kernel-include-regex 'k_trace<.*, false, [012]>' --output-format csv -d $OUT/pmc_$v -o pass -- python bench.py --config ${CFG:-C2} --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/pmc_$v.log 2>&1 || { echo "$v pmc failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
  python3 - "$OUT/pmc_$v" "$v" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.defaultdict(set)
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        kn = r["Kernel_Name"].rstrip()
        if not (kn.endswith("false>(bhrt_kparams)") or kn.split("<", 1)[-1].split(">")[0].split(",")[4].strip() == "false"): continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print(sys.argv[2], " ".join(f"{k}={acc[k]/max(len(n[k]),1):.4g}" for k in sorted(acc)))
PY
done
