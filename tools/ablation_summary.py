"""Summarise gpurun_out/ablation (tools/ablation_run.sh): VALU instructions per
ray-iteration and time per ray-iteration for the base build and each ablation."""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ablation"
rows = []
for j in sorted(glob.glob(os.path.join(src, "*.json"))):
    v = os.path.basename(j)[:-5]
    b = json.load(open(j))
    acc = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for p in glob.glob(os.path.join(src, f"pmc_{v}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].rstrip().endswith("false>(bhrt_kparams)"):
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]].add(r["Dispatch_Id"])
    per = {k: acc[k] / max(len(n[k]), 1) for k in acc}
    it = b["kernel"]["iterations_per_launch"]
    rows.append((v, 64 * per.get("SQ_INSTS_VALU", 0) / it,
                 64 * (per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_MUL_F64", 0)
                       + per.get("SQ_INSTS_VALU_ADD_F64", 0)) / it,
                 b["kernel"]["avg_ms"] * 1e9 / it, it))
base = {r[0]: r for r in rows}["base"]
print(f"{'variant':12s} {'VALU/it':>8s} {'dVALU':>7s} {'f64/it':>7s} {'ps/it':>7s} {'iters':>12s}")
for v, valu, f64, ps, it in rows:
    print(f"{v:12s} {valu:8.1f} {valu - base[1]:7.1f} {f64:7.1f} {ps:7.2f} {it:12.0f}")
