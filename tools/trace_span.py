"""Per-launch GPU time of a kernel from a rocprofv3 kernel trace (CSV), for launches that
overlap on several streams (bench.py --streams 2).

  python tools/trace_span.py gpurun_out/prof/run_kernel_trace.csv [--kernel 'k_trace<0, true, true, false, false, false>']

Prints the number of dispatches, their mean start..end duration (what rocprofv3 --stats
averages; overlapping launches double-count the overlap) and the union of their intervals
divided by the dispatch count (the GPU busy time per launch, bench.py's roofline duration).
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default=None,
                    help="kernel name (default: the k_trace instantiation with HUGE = false "
                         "that has the most GPU time in the trace)")
    ap.add_argument("--skip", type=int, default=0, help="leave out the first k dispatches "
                    "(bench.py's untimed warm-up frames)")
    ap.add_argument("--last", type=int, default=0, help="keep only the last k dispatches "
                    "(bench.py --no-host-path --steps k: its timed frames)")
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    if a.kernel is None:
        tot = {}
        for row in rows:
            k = row["Kernel_Name"]
            m = re.search(r"k_trace<([^>]*)>", k)
            if m and m.group(1).split(",")[4].strip() == "false":  # template arg 5 = HUGE
                tot[k] = tot.get(k, 0) + int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        a.kernel = max(tot, key=tot.get)
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if a.kernel in r["Kernel_Name"]]
    iv.sort()
    iv = iv[a.skip:]
    if a.last > 0:
        iv = iv[-a.last:]
    n = len(iv)
    mean = sum(e - s for s, e in iv) / n
    union, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    print(f"{a.kernel}: {n} dispatches, mean start..end {mean / 1e6:.4f} ms, "
          f"union of intervals / dispatches {union / n / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
