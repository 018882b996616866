#!/usr/bin/env python3
"""The GPU side of one trace_rays_batch call, from a rocprofv3 kernel + memory-copy trace.

  rocprofv3 --kernel-trace --memory-copy-trace -d D -o run --output-format csv -- \
      python3 tools/batch_probe.py
  python tools/batch_timeline.py D/.../run_kernel_trace.csv D/.../run_memory_copy_trace.csv

Prints every kernel dispatch and copy of one call (events are split into calls at idle gaps
longer than --gap ms; --call picks among those with trace kernels, default the last), in start order and
relative to the call's first event, then the union of busy time per kind: where the call's
wall time goes besides tracing (the first upload before any kernel, the last chunk's
download after the last kernel, gaps between them).
"""
import argparse
import csv
import re


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:50]


def union(iv):
    tot, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("copies")
    ap.add_argument("--gap", type=float, default=0.5, help="idle gap (ms) that separates calls")
    ap.add_argument("--call", type=int, default=-1, help="which call with trace kernels (-1: last)")
    ap.add_argument("--min-span", type=float, default=0.0,
                    help="only calls at least this long (ms): skips trace_ray calls after a batch")
    a = ap.parse_args()
    ev = []
    with open(a.kernels) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K",
                       short(r["Kernel_Name"])))
    with open(a.copies) as f:
        for r in csv.DictReader(f):
            d = r.get("Direction") or r.get("Kind") or "copy"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C",
                       d + (f" {int(r['Bytes']) / 1e6:.1f} MB" if r.get("Bytes") else "")))
    ev.sort()
    # split into calls at idle gaps; keep the last call
    calls, cur, end = [], [], None
    for e in ev:
        if end is not None and e[0] - end > a.gap * 1e6:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = e[1] if end is None else max(end, e[1])
    calls.append(cur)
    calls = [c for c in calls if any(n.startswith("k_trace") for _, _, _, n in c) and
             (max(e for _, e, _, _ in c) - c[0][0]) / 1e6 >= a.min_span]
    last = calls[a.call]
    t0 = last[0][0]
    for s, e, k, n in last:
        print(f"{(s - t0) / 1e6:8.3f} .. {(e - t0) / 1e6:8.3f} ms  {(e - s) / 1e6:7.3f}  {k} {n}")
    span = (max(e for _, e, _, _ in last) - t0) / 1e6
    kb = union([(s, e) for s, e, k, _ in last if k == "K"]) / 1e6
    cb = union([(s, e) for s, e, k, _ in last if k == "C"]) / 1e6
    ab = union([(s, e) for s, e, _, _ in last]) / 1e6
    print(f"call: span {span:.3f} ms, kernels busy {kb:.3f}, copies busy {cb:.3f}, "
          f"any busy {ab:.3f}, idle {span - ab:.3f} ms ({len(calls)} calls in the trace)")


if __name__ == "__main__":
    main()
