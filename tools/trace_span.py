"""Per-launch GPU time of a kernel from a rocprofv3 kernel trace (CSV), for launches that
overlap on several streams (bench.py --streams 2).

  python tools/trace_span.py gpurun_out/prof/run_kernel_trace.csv [--kernel 'k_trace<0, true, true, false, false, false>']

Prints the number of dispatches, their mean start..end duration (what rocprofv3 --stats
averages; overlapping launches double-count the overlap) and the union of their intervals
divided by the dispatch count (the GPU busy time per launch, bench.py's roofline duration).
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_trace<0, true, true, false, false, false>")
    ap.add_argument("--skip", type=int, default=0, help="leave out the first k dispatches "
                    "(bench.py's untimed warm-up frames)")
    a = ap.parse_args()
    iv = []
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            if a.kernel in row["Kernel_Name"]:
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    iv.sort()
    iv = iv[a.skip:]
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
