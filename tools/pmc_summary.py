"""Summarise rocprofv3 --pmc passes of tools/pmc.sh into profiles/pmc_<CFG>.json.

HBM bytes per launch follow MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced stream, so it is doubled (the
trace kernel's init-table reads are 8-byte-per-lane loads, for which the guide gives no
calibration: both the raw and the corrected figure are recorded)."""
import collections
import csv
import glob
import json
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
cfg = sys.argv[2] if len(sys.argv) > 2 else "C2"
per = collections.defaultdict(list)
for p in sorted(glob.glob(f"{src}/p*/pass_counter_collection.csv")):
    acc = collections.defaultdict(float)
    for row in csv.DictReader(open(p)):
        # the hot instantiation only (HUGE = false); the redo launch is normally empty
        m = re.search(r"k_trace<([^>]*)>", row.get("Kernel_Name", ""))
        if not m or m.group(1).split(",")[4].strip() != "false":   # template arg 5 = HUGE
            continue
        acc[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (disp, name), v in acc.items():
        per[name].append(v)
avg = {k: sum(v) / len(v) for k, v in per.items()}
out = {"config": cfg, "kernel": "k_trace (hot instantiation, HUGE=false)", "counters_per_launch": avg}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    out["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
    out["write_bytes"] = avg["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = int(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024)
if "GRBM_GUI_ACTIVE" in avg:
    out["note"] = "effective clock = GRBM_GUI_ACTIVE / 8 / kernel time"
json.dump(out, open(f"profiles/pmc_{cfg}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
