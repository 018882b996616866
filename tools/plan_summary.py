#!/usr/bin/env python3
"""Load balance and predicted scaling efficiency of the N-GPU plans from one-GPU shard timings.

  python tools/plan_summary.py gpurun_out/plan_shards.jsonl [--out profiles/...txt]

Input: bench.py lines from tools/plan_shards.sh -- per config the N = 1 line (plan_gpus 1) and
one line per shard k of the N-GPU plan (plan_gpus N, shard k). Each shard line's ms_per_step is
what rank k of the N-GPU run spends per frame on tracing (the RCCL gather of the rgba8 image,
overlapped with the next frame, is not in it). The N-GPU run's value is the frame's rays / the
slowest rank's time, so

  load balance      max_k T_k / mean_k T_k
  predicted value   sum_k rays_k / max_k T_k                          (Mrays/s, whole job)
  efficiency        predicted value / (N x the N = 1 line's value)    (weak: C1-C3, C5;
                                                                       strong: C4)
"""
import argparse
import json
import sys
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("jsonl")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    base, shards = {}, defaultdict(dict)
    with open(a.jsonl) as f:
        for line in f:
            line = line.strip()
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            cfg = r["config"]["workload"].split(":")[0]
            n = r["config"].get("plan_gpus", 1)
            if n == 1:
                base[cfg] = r
            else:
                shards[(cfg, n)][r["config"]["shard"]] = r
    out = []
    for (cfg, n), by in sorted(shards.items()):
        ks = sorted(by)
        t = [by[k]["ms_per_step"] for k in ks]
        rays = [by[k]["config"]["rays_per_frame"] for k in ks]
        kern = [by[k]["kernel"]["avg_ms"] for k in ks]
        value = sum(rays) / (max(t) * 1e-3) / 1e6
        b = base.get(cfg)
        eff = value / (n * b["value"]) if b else None
        kind = "strong" if b and b["scaling"] == "strong" else "weak"
        out.append(f"{cfg} plan {n} GPUs ({len(ks)} shards timed): "
                   f"{by[ks[0]]['config']['width']}x{by[ks[0]]['config']['height']}, "
                   f"rays/shard {min(rays)}..{max(rays)}")
        for k, tk, kk, rk in zip(ks, t, kern, rays):
            out.append(f"  shard {k}: {tk:8.3f} ms/frame (trace kernel span {kk:.3f} ms), "
                       f"{rk / tk / 1e3:9.1f} Mrays/s")
        mean = sum(t) / len(t)
        out.append(f"  load balance max/mean {max(t) / mean:.4f} (max {max(t):.3f}, mean "
                   f"{mean:.3f}, min {min(t):.3f} ms)")
        if b:
            out.append(f"  N=1 line: {b['value']:.1f} Mrays/s, {b['ms_per_step']:.3f} ms/frame "
                       f"({b['config']['width']}x{b['config']['height']}, "
                       f"{b['config']['rays_per_frame']} rays)")
            out.append(f"  predicted N={n}: {value:.1f} Mrays/s whole job, {kind} efficiency "
                       f"{eff:.3f}")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
