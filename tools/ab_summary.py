#!/usr/bin/env python3
"""Mean value per variant of tools/ab.sh output files (lines: CFG VARIANT ROUND Mrays/s ms).

  python tools/ab_summary.py gpurun_out/<tag>/ab_*.txt"""
import collections
import sys

for path in sys.argv[1:]:
    d = collections.defaultdict(list)
    for line in open(path):
        p = line.split()
        if len(p) >= 5:
            try:
                d[p[1]].append(float(p[3]))
            except ValueError:
                pass
    print(f"## {path}")
    base = None
    for k, v in d.items():
        m = sum(v) / len(v)
        base = base or m
        print(f"   {k:40s} {m:10.1f}  {m / base - 1:+7.1%}  {v}")
