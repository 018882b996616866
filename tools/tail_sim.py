#!/usr/bin/env python3
"""Replay of k_trace's wave scheduler over a frame's per-ray iteration counts (numpy).

  python tools/tail_sim.py gpurun_out/a/steps.npz --config C4 --plan 8 --shard 0 \
      [--policy current exact prefetch tail16 ...] [--frames 12 --streams 4]

What is modelled ("wave granularity"):
  * the shard's rays in the kernel's claim order: 64-ray tiles (8x8, 16x4 or 32x2, the first
    that divides the shard, bhrt_api.c claim_tiles) dealt in 64-id blocks round robin over 16
    queues (geodesic.hip queue_ray); a tile's cost is its longest ray's iterations (a wave runs
    an iteration while any lane needs it) plus a set-up cost per refill;
  * 4 waves per SIMD, 4 SIMDs per CU, 256 CUs; a workgroup (4 waves, one per SIMD) is a slot
    that frees only when all its waves have exited; several launches in flight (--streams):
    launch k + streams waits for launch k, and a launch's workgroups take slots as they free;
  * per-wave speed when k waves share a SIMD: min(s1, 4 / k) iterations per time unit (4 waves
    issue one iteration each per unit; a lone wave is latency-bound at s1);
  * claim policies (one returning atomic per claim costs --claim-lat units of stall unless it
    was issued ahead):
      current   the shipped guided claim: a claim takes the queue's remainder as the wave last
                saw it (size - hi) >> shift tiles, shift from waves / queues -- so every wave's
                FIRST claim, made with hi = 0, takes size / (waves per queue): the launch is
                statically partitioned at its start;
      exact     one tile per claim (claim_div 0);
      gss       a claim takes the queue's true remainder / (waves per queue) (read at claim);
      prefetch  one tile per claim, the next claim issued a trip ahead (latency hidden);
      tail<k>   current, but once the queue's remainder is below the resident lanes the wave
                refills when k lanes are idle (lane refill: a tile's rays start as lanes free).
Prints per policy: the frame time (time units per frame in steady state) and its ratio to the
ideal (total iteration work / full-chip throughput).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

CUS, SIMDS, WPS = 256, 4, 4          # CUs, SIMDs per CU, waves per SIMD
WG_SLOTS = CUS * WPS                  # workgroups of 4 waves resident at once
NQ = 16


def shard_iters(z, config, plan, shard):
    from bhrt import abi, configs
    c = configs.CONFIGS[config]
    st = z[f"{config}_steps"].astype(np.int64)
    res = z[f"{config}_result"]
    it = st + np.isin(res, (abi.RAY_HORIZON, abi.RAY_MAX_DISTANCE))
    p = c.frame(plan)
    if p.shards > 1:
        rows = np.arange(p.height)
        it = it[((rows // p.row_block) % p.shards) == shard]
    return it


def tiles_of(it):
    """per-ray iterations [rows, W] -> per-tile (64 rays) iteration lists in claim order"""
    H, W = it.shape
    for tw, th in ((8, 8), (16, 4), (32, 2)):
        if W % tw == 0 and H % th == 0:
            t = it.reshape(H // th, th, W // tw, tw).transpose(0, 2, 1, 3).reshape(-1, 64)
            return t
    return it.reshape(-1)[: (it.size // 64) * 64].reshape(-1, 64)


class Launch:
    def __init__(self, tiles, policy, waves):
        self.tiles = tiles                       # [ntiles, 64]
        self.tmax = tiles.max(axis=1)
        n = len(tiles)
        self.q = [list(range(q, n, NQ)) for q in range(NQ)]   # tile ids per queue
        self.head = [0] * NQ
        self.size = [len(x) for x in self.q]
        self.policy = policy
        self.waves = waves
        self.shift_tiles = max(1, waves // NQ)   # claim = remainder / (waves per queue)
        self.left = n

    def claim(self, w, st):
        """next tile for wave state st (dict); returns (tile id or None, stalled)"""
        # hand out from the wave's own block first
        if st["lo"] < st["hi"]:
            t = self.q[st["cur"]][st["lo"]]
            st["lo"] += 1
            return t, False
        pol = self.policy
        while st["moves"] < NQ:
            q = st["cur"]
            rem_seen = self.size[q] - st["hi"]
            rem_true = self.size[q] - self.head[q]
            if pol.startswith("current") or pol.startswith("tail"):
                c = 1 if st["hopped"] else max(1, -(-rem_seen // self.shift_tiles))
            elif pol == "gss":
                c = 1 if st["hopped"] else max(1, -(-rem_true // self.shift_tiles))
            else:
                c = 1
            base = self.head[q]
            if base < self.size[q]:
                self.head[q] = base + c
                e = min(base + c, self.size[q])
                st["lo"], st["hi"] = base + 1, e
                self.left -= 1
                return self.q[q][base], not (pol == "prefetch")
            st["moves"] += 1
            st["cur"] = (q + 1) % NQ
            st["hi"] = 0
            st["hopped"] = True
        return None, False


def simulate(tiles, policy, frames, streams, s1, claim_lat, setup, dt=0.25):
    """steady-state time per frame (time units: one iteration of a wave sharing its SIMD with 3)"""
    waves_per_launch = WG_SLOTS * 4
    tail_k = int(policy[4:]) if policy.startswith("tail") else None
    # slot table: WG slot -> (launch, wg index) or free
    slot_launch = -np.ones(WG_SLOTS, dtype=np.int64)
    # wave arrays (per resident wave position: slot*4 + simd)
    nwp = WG_SLOTS * 4
    busy = np.zeros(nwp)          # remaining work units of the current tile (or lane pool)
    stall = np.zeros(nwp)         # remaining stall (claim latency)
    alive = np.zeros(nwp, dtype=bool)
    simd_of = (np.arange(nwp) // 4 // WPS) * SIMDS + (np.arange(nwp) % 4)   # CU*4 + simd
    launches, states = {}, {}
    pending = []                  # (launch id, next wg index to dispatch)
    started = 0
    done_t = {}
    t = 0.0
    lanes = {}                    # tail policy: per wave, remaining iterations of each lane

    def start_launch(k):
        launches[k] = Launch(tiles, policy, waves_per_launch)
        pending.append([k, 0])

    for k in range(min(streams, frames)):
        start_launch(k)
    started = min(streams, frames)
    wave_owner = -np.ones(nwp, dtype=np.int64)
    wave_state = [None] * nwp
    steps = 0
    while True:
        # dispatch pending workgroups into free slots (oldest launch first)
        free = np.flatnonzero(slot_launch < 0)
        fi = 0
        for p in pending:
            k, nxt = p
            while nxt < WG_SLOTS and fi < len(free):
                sl = free[fi]
                fi += 1
                slot_launch[sl] = k
                for j in range(4):
                    wp = sl * 4 + j
                    wave_owner[wp] = k
                    wave_state[wp] = {"lo": 0, "hi": 0, "cur": (nxt * 4 + j) % NQ, "moves": 0,
                                      "hopped": False, "need": True}
                    alive[wp] = True
                    busy[wp] = 0.0
                    stall[wp] = 0.0
                nxt += 1
            p[1] = nxt
        pending[:] = [p for p in pending if p[1] < WG_SLOTS]
        # claims for waves that need work
        need = np.flatnonzero(alive & (busy <= 0) & (stall <= 0))
        for wp in need:
            k = wave_owner[wp]
            L = launches[k]
            st = wave_state[wp]
            if tail_k is not None and wp in lanes:
                pass
            tid, stalled = L.claim(wp, st)
            if tid is None:
                alive[wp] = False
                lanes.pop(wp, None)
                continue
            busy[wp] = L.tmax[tid] + setup
            if stalled:
                stall[wp] = claim_lat
        # a workgroup's slot frees when its 4 waves are gone
        occ = alive.reshape(WG_SLOTS, 4).any(axis=1)
        fin = (~occ) & (slot_launch >= 0)
        if fin.any():
            for sl in np.flatnonzero(fin):
                slot_launch[sl] = -1
        # launch completion
        for k in list(launches):
            if k in done_t:
                continue
            if not any(p[0] == k for p in pending) and not (alive & (wave_owner == k)).any():
                done_t[k] = t
                if started < frames:
                    start_launch(started)
                    started += 1
        if len(done_t) == frames:
            break
        # advance time
        comp = alive & (stall <= 0) & (busy > 0)
        k_simd = np.bincount(simd_of[comp], minlength=CUS * SIMDS)
        sp = np.minimum(s1, 4.0 / np.maximum(k_simd[simd_of], 1))
        busy[comp] -= sp[comp] * dt
        stall[alive & (stall > 0)] -= dt
        t += dt
        steps += 1
        if steps > 10_000_000:
            raise RuntimeError("no progress")
    # steady state: frames after the first `streams` completions
    ts = sorted(done_t.values())
    k0 = min(streams, frames - 2)
    return (ts[-1] - ts[k0]) / (frames - 1 - k0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("steps")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--plan", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--policy", nargs="+", default=["current", "exact", "gss", "prefetch"])
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--s1", type=float, default=2.0, help="lone-wave speed (x the 4-wave rate)")
    ap.add_argument("--claim-lat", type=float, default=2.0, help="claim stall (iterations)")
    ap.add_argument("--setup", type=float, default=3.0, help="refill set-up (iterations)")
    a = ap.parse_args()
    z = np.load(a.steps)
    it = shard_iters(z, a.config, a.plan, a.shard)
    tiles = tiles_of(it)
    ideal = (tiles.max(axis=1).sum() + a.setup * len(tiles)) / (WG_SLOTS * 4)
    ideal_lanes = it.sum() / (WG_SLOTS * 4 * 64)
    print(f"{a.config} plan {a.plan} shard {a.shard}: {it.size} rays, {len(tiles)} tiles, mean "
          f"{it.mean():.2f} iterations/ray, tile max mean {tiles.max(axis=1).mean():.2f}; "
          f"ideal frame {ideal:.1f} units (tile-max work), {ideal_lanes:.1f} (lane work)")
    for pol in a.policy:
        f = simulate(tiles, pol, a.frames, a.streams, a.s1, a.claim_lat, a.setup)
        print(f"  {pol:10s} {f:8.1f} units/frame  x{f / ideal:.3f} of ideal")


if __name__ == "__main__":
    main()
