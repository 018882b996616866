#!/usr/bin/env python3
"""Where a frame's GPU time goes beside the trace kernel, from a rocprofv3 kernel trace (CSV).

  python tools/frame_timeline.py gpurun_out/prof/run_kernel_trace.csv [--skip 3]

A frame of bench.py is: two control-block memsets (hipMemsetAsync -> fill kernels), the hot
k_trace launch (HUGE = false), the redo launch (HUGE = true, normally finds an empty list) and
k_colour. The frames are delimited by the hot k_trace dispatches (after --skip warm-up
frames). Printed per frame: every kernel's dispatches and mean / total duration, the union of
all dispatch intervals (GPU busy), and the window from the first frame's first dispatch to the
last dispatch's end -- window - busy is GPU idle time (launch latency, gaps between
dependent dispatches). Run it on a --streams 1 trace for the serial per-frame cost.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=0, help="warm-up frames to leave out")
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(f)]
    rows.sort()

    def hot(n):
        m = re.match(r"k_trace<([^>]*)>", n)
        return m and m.group(1).split(",")[4].strip() == "false"

    starts = [i for i, r in enumerate(rows) if hot(r[2])]
    if len(starts) <= a.skip:
        raise SystemExit("not enough frames")
    # a frame owns the dispatches from just after the previous hot launch's trailing work: take
    # the first dispatch of frame k as the one right after frame k-1's last non-memset kernel;
    # simpler and exact for --streams 1: the memsets immediately precede the hot launch
    first = starts[a.skip]
    i0 = first
    while i0 > 0 and "k_" not in rows[i0 - 1][2]:
        i0 -= 1
    sel = rows[i0:]
    frames = len(starts) - a.skip
    by = defaultdict(list)
    for s, e, n in sel:
        by[n].append(e - s)
    union, cs, ce = 0, None, None
    for s, e, _ in sel:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    window = max(e for _, e, _ in sel) - sel[0][0]
    print(f"{frames} frames (after {a.skip} skipped), {len(sel)} dispatches")
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:60s} {len(d) / frames:5.2f}/frame  mean {sum(d) / len(d) / 1e3:9.2f} us  "
              f"per frame {sum(d) / frames / 1e3:9.2f} us")
    print(f"  GPU busy (union) per frame {union / frames / 1e3:9.2f} us; window per frame "
          f"{window / frames / 1e3:9.2f} us; idle per frame {(window - union) / frames / 1e3:9.2f} us")


if __name__ == "__main__":
    main()
