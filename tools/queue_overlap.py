"""Which hardware queue / stream each of the last frames' kernels ran on, and how much they
overlapped (rocprofv3 --kernel-trace --output-format csv). Usage:
    python tools/queue_overlap.py <kernel_trace.csv> [last_n_trace_kernels]"""
import csv
import sys
from collections import Counter, defaultdict


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tr = [r for r in rows if "k_trace" in r["Kernel_Name"]]
    if not tr:
        print("no k_trace kernels")
        return
    t_first = int(tr[-last]["Start_Timestamp"]) if len(tr) >= last else int(tr[0]["Start_Timestamp"])
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t_first]
    kt = [r for r in win if "k_trace" in r["Kernel_Name"]]
    print(f"{len(kt)} trace kernels, {len(win)} kernels in the window")
    by = Counter((r.get("Queue_Id"), r.get("Stream_Id")) for r in kt)
    for (q, s), n in sorted(by.items()):
        print(f"  queue {q} stream {s}: {n} trace kernels")
    other = Counter((r["Kernel_Name"][:60], r.get("Queue_Id"), r.get("Stream_Id"))
                    for r in win if "k_trace" not in r["Kernel_Name"])
    for (k, q, s), n in sorted(other.items()):
        print(f"  other: {k} queue {q} stream {s}: {n}")
    ev = []
    for r in kt:
        ev.append((int(r["Start_Timestamp"]), 1))
        ev.append((int(r["End_Timestamp"]), -1))
    ev.sort()
    t0, t1 = ev[0][0], ev[-1][0]
    busy = defaultdict(int)
    cur, prev = 0, t0
    for t, d in ev:
        busy[cur] += t - prev
        cur += d
        prev = t
    span = t1 - t0
    print(f"span {span / 1e6:.3f} ms = {span / 1e6 / len(kt):.4f} ms per trace kernel; "
          f"mean duration {sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in kt) / len(kt) / 1e6:.4f} ms")
    for k in sorted(busy):
        print(f"  {k} trace kernels running: {busy[k] / span:.3f} of the span")
    # gap from a kernel's end to the next start on the same stream
    last_end = {}
    gaps = defaultdict(list)
    for r in sorted(kt, key=lambda r: int(r["Start_Timestamp"])):
        s = r.get("Stream_Id")
        if s in last_end:
            gaps[s].append(int(r["Start_Timestamp"]) - last_end[s])
        last_end[s] = int(r["End_Timestamp"])
    for s, g in sorted(gaps.items()):
        g.sort()
        print(f"  stream {s}: end->next start median {g[len(g) // 2] / 1e3:.1f} us, max {g[-1] / 1e3:.1f} us")


if __name__ == "__main__":
    main()
