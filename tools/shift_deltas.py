#!/usr/bin/env python3
"""How large are the angle shifts of the C2 trace loop (geodesic.hip shift_or_eval)?

The a = 0 RK4 iteration takes six sin/cos by angle addition from a nearby known angle: stage 2,
3, 4 of ray_derivatives' theta (= state[1]) from stage 1 (delta = h/2 k1, h/2 k2, h k3 of
component 1), and the advance of state[1], [2], [3] by one step. The polynomials of a shift are
fitted to |delta| <= T (the fast path); a lane beyond T takes the wide shift, and a wave runs that
branch whenever ANY of its lanes needs it. This replays the C2 scene's RK4 in numpy (literal
ray_derivatives, raytracer.c:44-154; every ray run to its oracle step count) on a camera-B frame
and reports, per site and threshold T, the fraction of lane evaluations beyond T and the fraction
of 8x8-tile "waves" (a wave's 64 lanes = one claim tile) with any lane beyond T.

  python tools/shift_deltas.py [W H]   (default 480x270; CPU only)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bhrt import abi, configs  # noqa: E402
import oracle as orc  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (480, 270)
c = configs.CONFIGS["C2"]
bh, dk, cfg = c.scene()
cam = configs.camera("B")
rays = configs.camera_rays(cam, W, H)
ref = orc.oracle().trace_rays(rays, bh, dk, cfg, c.method, c.flags)
# iterations each ray executes: steps (+1 for HORIZON / MAX_DISTANCE exits; DISK: steps)
iters = ref["steps"].astype(np.int64) + np.isin(ref["result"], (abi.RAY_HORIZON,
                                                                abi.RAY_MAX_DISTANCE))
M, rs, dt = bh.mass, bh.schwarzschild_radius, cfg.time_step
o = rays["origin"][0]
r0 = float(np.sqrt(o @ o))
th0, ph0 = np.arccos(o[2] / r0), np.arctan2(o[1], o[0]) % (2 * np.pi)
d = rays["direction"] / np.linalg.norm(rays["direction"], axis=1)[:, None]
st, ct, sp, cp = np.sin(th0), np.cos(th0), np.sin(ph0), np.cos(ph0)
vr = st * cp * d[:, 0] + st * sp * d[:, 1] + ct * d[:, 2]
vth = (ct * cp * d[:, 0] + ct * sp * d[:, 1] - st * d[:, 2]) / r0
vph = (-sp * d[:, 0] + cp * d[:, 1]) / (r0 * st)
rm = max(r0, rs + 1e-10)
g_tt, g_rr, g_hh = -(1 - rs / rm), 1 / (1 - rs / rm), rm * rm
vt = np.sqrt(np.maximum(-(g_rr * vr * vr + g_hh * vth * vth + g_hh * vph * vph) / g_tt, 0.0))
n = len(rays)
y = np.stack([np.zeros(n), np.full(n, r0), np.full(n, th0), np.full(n, ph0), vt, vr])


def derivs(s):
    r, th, v_r, v_th, v_ph = s[0].copy(), s[1], s[3], s[4], s[5]
    out = np.empty_like(s)
    out[0], out[1], out[2] = v_r, v_th, v_ph
    sn = np.sin(th)
    r = np.where(r <= rs * 1.5, rs * 1.5, r)
    sn = np.where(np.abs(sn) < 0.01, np.where(sn >= 0, 0.01, -0.01), sn)
    with np.errstate(all="ignore"):
        f = 1.0 - rs / r
        out[3] = -M / (r * r * f) * f + r * v_th * v_th + r * sn * sn * v_ph * v_ph
        out[4] = -2.0 * v_r * v_th / r + sn * np.cos(th) * v_ph * v_ph
        out[5] = -2.0 * v_r * v_ph / r - 2.0 * v_th * v_ph * np.cos(th) / sn
    out[3:] = np.clip(np.nan_to_num(out[3:], nan=0.0, posinf=0.0, neginf=0.0), -10, 10)
    return out


sites = ("stage2", "stage3", "stage4", "adv_y1", "adv_y2", "adv_y3")
TS = (1 / 16, 1 / 32, 1 / 64, 1 / 128)
lane_over = {s: np.zeros(len(TS)) for s in sites}
wave_over = {s: np.zeros(len(TS)) for s in sites}
lane_evals = wave_evals = 0
# tiles of 8x8 pixels as waves
px, py = np.arange(n) % W, np.arange(n) // W
tile = (py // 8) * ((W + 7) // 8) + px // 8
ntile = tile.max() + 1
hmax = {}
for k in range(int(iters.max())):
    alive = iters > k
    if not alive.any():
        break
    r = y[1]
    h = np.where(r < rs * 2.5, min(dt * 0.001, 0.1), np.where(r < rs * 5, min(dt * 0.01, 0.1),
                 np.where(r < rs * 15, min(dt * 0.1, 0.1), min(dt, 0.1))))
    k1 = derivs(y)
    k2 = derivs(y + 0.5 * h * k1)
    k3 = derivs(y + 0.5 * h * k2)
    k4 = derivs(y + h * k3)
    ynew = y + h * (k1 + 2 * k2 + 2 * k3 + k4) / 6.0
    deltas = {"stage2": 0.5 * h * k1[1], "stage3": 0.5 * h * k2[1], "stage4": h * k3[1],
              "adv_y1": ynew[1] - y[1], "adv_y2": ynew[2] - y[2], "adv_y3": ynew[3] - y[3]}
    lane_evals += int(alive.sum())
    tiles_alive = np.bincount(tile[alive], minlength=ntile) > 0
    wave_evals += int(tiles_alive.sum())
    for s, dl in deltas.items():
        a = np.abs(dl)
        for j, T in enumerate(TS):
            over = alive & (a > T)
            lane_over[s][j] += over.sum()
            wave_over[s][j] += (np.bincount(tile[over], minlength=ntile) > 0).sum()
    y = np.where(alive, ynew, y)
print(f"C2 camera B {W}x{H}: {lane_evals} lane-iterations, {wave_evals} tile-iterations")
print("site      " + "  ".join(f"lane>{T:.4g} wave>{T:.4g}" for T in TS))
for s in sites:
    print(f"{s:8s}  " + "  ".join(f"{lane_over[s][j] / lane_evals:9.5f} {wave_over[s][j] / wave_evals:9.5f}"
                                   for j in range(len(TS))))
