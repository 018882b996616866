#!/usr/bin/env python3
"""Why wave slots sit empty, from a tools/wave_stamps.py record.

  python tools/stamp_occupancy.py gpurun_out/<tag>/stamps_C4_p8_s0_x4.npz

For 0.5 us bins over the timed frames: resident trace waves (all launches) and the waves of
already-started launches that have not started yet ("pending"). Prints the fraction of time
under 75% of the 4096 resident waves, how often waves were pending then (pending with free
slots = workgroup granularity: a 4-wave workgroup needs four free wave slots on one CU; none
pending = every launch in flight is fully dispatched and the next frame's launch still waits
behind its stream), and the wave start rate while waves were pending.
"""
import sys

import numpy as np


def main(path):
    z = np.load(path)
    ks = sorted([k for k in z.files if k.startswith("slot")], key=lambda k: int(k[4:]))
    recs = [z[k].astype(np.int64) for k in ks]
    recs.sort(key=lambda r: r[:, 0].min())
    lo = min(r[:, 0].min() for r in recs)
    hi = max(r[:, 1].max() for r in recs)
    T = np.arange(lo, hi, 50)
    occ = np.zeros(len(T))
    pend = np.zeros(len(T))
    for r in recs:
        s, e = r[:, 0], r[:, 1]
        d = np.zeros(len(T) + 1)
        np.add.at(d, np.searchsorted(T, s), 1)
        np.add.at(d, np.searchsorted(T, e), -1)
        occ += np.cumsum(d)[:-1]
        ss = np.sort(s)
        notyet = len(ss) - np.searchsorted(ss, T, side="right")
        pend += np.where((T >= s.min()) & (T < e.max()), notyet, 0)
    low = occ < 0.75 * 4096
    print(f"{path}: under 75% resident {low.mean() * 100:.1f}% of the time; waves pending then "
          f"{(pend[low] > 0).mean() * 100:.1f}% of it; mean resident {occ.mean():.0f}")
    st = np.sort(np.concatenate([r[:, 0] for r in recs]))
    bins = np.arange(lo, hi, 500)
    cnt = np.histogram(st, bins)[0]
    mid = np.minimum(np.searchsorted(T, bins[:-1]), len(T) - 1)
    sel = (pend[mid] > 500) & (occ[mid] < 3500)
    if sel.any():
        print(f"  wave starts per 5 us while > 500 waves pending and < 3500 resident: "
              f"{cnt[sel].mean():.0f} ({sel.sum()} windows)")


if __name__ == "__main__":
    main(sys.argv[1])
