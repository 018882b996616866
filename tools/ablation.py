"""Cost accounting for the trace loop: builds libbhrt variants that each REMOVE one piece of
per-iteration work (results become wrong -- these are for accounting only, never shipped)
into raytracing-engine-in-c_amd/ab/libbhrt_x_<name>.so. tools/ablation_run.sh then measures
VALU instructions per ray-iteration (rocprofv3 PMC) and kernel time for each.

    python tools/ablation.py            # build the variants (here, no GPU needed)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raytracing-engine-in-c_amd", "csrc")
AB = os.path.join(ROOT, "raytracing-engine-in-c_amd", "ab")

# name -> list of (old, new) source substitutions in geodesic.hip
ABLATIONS = {
    "chain": [("        if (SPIN0)  // spin != 0: ray_derivatives never takes sin/cos of state[1] (:131-138)\n            trig_advance(tr.a, R.y[1], R.s1, R.c1, hc);", ""),
              ("        trig_advance(tr.a, R.y[1], R.s1, R.c1, hc);", ""),
              ("        trig_advance(a2, R.y[2], R.s2, R.c2, hc);", ""),
              ("        trig_advance(a3, R.y[3], R.s3, R.c3, hc);", "")],
    "stageshift": [("} else if (!sincos_shift(tr.a, tr.s, tr.c, y[1], st, ct)) {",
                    "} else if (st = tr.s, ct = tr.c, false) {")],
    "div": [("__device__ __forceinline__ double rcp_nr(double b) {",
             "__device__ __forceinline__ double rcp_nr(double b) {\n    return __builtin_amdgcn_rcp(b);"),
            ("__device__ __forceinline__ double div_nr(double a, double b, double yb) {",
             "__device__ __forceinline__ double div_nr(double a, double b, double yb) {\n    return a * yb;")],
    "clamp": [("    if (!finite) {", "    if (false) {"),
              ("    for (int i = 3; i < 6; i++) d[i] = fmin(fmax(d[i], -10.0), 10.0);", "    for (int i = 3; i < 3; i++) {}")],
    "disk": [("    if (fabs(den) < kEps) return false;", "    return false;")],
    "dist": [("    R.dist += len3(x - ox, y - oy, z - oz);",
              "    R.dist += (x - ox) * (x - ox) + (y - oy) * (y - oy) + (z - oz) * (z - oz);")],
}


def main():
    os.makedirs(AB, exist_ok=True)
    base = open(os.path.join(CSRC, "geodesic.hip")).read()
    for name, subs in ABLATIONS.items():
        src, hits = base, 0
        for old, new in subs:
            if old in src:
                src, hits = src.replace(old, new), hits + 1
        if hits == 0:
            sys.exit(f"ablation {name}: no substitution matched")
        path = os.path.join(CSRC, f"_x_{name}.hip")
        open(path, "w").write(src)
        obj = os.path.join(CSRC, "build", f"x_{name}")
        os.makedirs(obj, exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-std=c++17", "-fvisibility=hidden", "-DBHRT_CONTRACT=1", "-c", path,
                        "-o", os.path.join(obj, "geodesic.o")], check=True, cwd=CSRC)
        os.remove(path)
        for f in ("particles.o", "bhrt_api.o", "particles_host.o", "kerr_helpers.o"):
            if not os.path.exists(os.path.join(CSRC, f)):
                sys.exit("build the library first (make -C raytracing-engine-in-c_amd/csrc)")
        objs = [os.path.join(obj, "geodesic.o")] + [os.path.join(CSRC, f) for f in
                                                     ("particles.o", "bhrt_api.o",
                                                      "particles_host.o", "kerr_helpers.o")]
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(AB, f"libbhrt_x_{name}.so"), *objs, "-lm"], check=True)
        print("built", name, f"({hits}/{len(subs)} substitutions)")


if __name__ == "__main__":
    main()
