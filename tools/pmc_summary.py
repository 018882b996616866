"""Summarise rocprofv3 --pmc passes of tools/pmc.sh into a pmc_<CFG>.json (profiles/).

  python tools/pmc_summary.py <pass dir> <CFG> [<out.json>]

HBM bytes per launch follow MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream, so it is doubled (the
trace kernel's init-table reads are 8-byte-per-lane loads, for which the guide gives no
calibration: both the raw and the corrected figure are recorded).

Issued FP64 work per launch = (2 FMA + MUL + ADD + TRANS) f64 wave instructions x 64 lanes
(an upper bound: lanes masked off by EXEC are counted too). VALU issue busy = VALU wave
instructions x 4 cycles (one wave64 instruction on a 16-lane-wide FP64 SIMD slot) / (1024
SIMDs x the kernel's cycles, GRBM_GUI_ACTIVE / 8 XCDs)."""
import collections
import csv
import glob
import json
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
cfg = sys.argv[2] if len(sys.argv) > 2 else "C2"
dst = sys.argv[3] if len(sys.argv) > 3 else f"profiles/pmc_{cfg}.json"
per = collections.defaultdict(list)
names = set()
for p in sorted(glob.glob(f"{src}/p*/pass_counter_collection.csv")):
    acc = collections.defaultdict(float)
    for row in csv.DictReader(open(p)):
        # the hot instantiation only (HUGE = false); the redo launch is normally empty
        m = re.search(r"k_trace<([^>]*)>", row.get("Kernel_Name", ""))
        if not m or m.group(1).split(",")[4].strip() != "false":   # template arg 5 = HUGE
            continue
        names.add(m.group(0))
        acc[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (disp, name), v in acc.items():
        per[name].append(v)
avg = {k: sum(v) / len(v) for k, v in per.items()}
out = {"config": cfg, "kernel": "k_trace (hot instantiation, HUGE=false)",
       "instantiations": sorted(names), "counters_per_launch": avg}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    out["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
    out["write_bytes"] = avg["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = int(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024)
f64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
       "SQ_INSTS_VALU_TRANS_F64")
if all(k in avg for k in f64):
    out["issued_fp64_flops_per_launch"] = 64 * (2 * avg[f64[0]] + avg[f64[1]] + avg[f64[2]] +
                                                avg[f64[3]])
    out["fp64_share_of_valu"] = sum(avg[k] for k in f64) / avg["SQ_INSTS_VALU"]
if "GRBM_GUI_ACTIVE" in avg:
    cycles = avg["GRBM_GUI_ACTIVE"] / 8
    out["kernel_cycles"] = cycles
    if "SQ_INSTS_VALU" in avg:
        out["valu_issue_busy"] = round(avg["SQ_INSTS_VALU"] * 4 / (1024 * cycles), 4)
    out["note"] = "effective clock = GRBM_GUI_ACTIVE / 8 / kernel time"
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
