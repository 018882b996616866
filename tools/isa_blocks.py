#!/usr/bin/env python3
"""Basic blocks of one kernel in a hipcc -S listing: label, instruction count, VALU / FP64 /
SALU / memory counts and the branch at the end -- to find and read the hot loop body.

usage: python tools/isa_blocks.py listing.s <kernel-name-substring> [--min N] [--dump LABEL]"""
import re, sys

path, key = sys.argv[1], sys.argv[2]
mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0] and l.split(":")[0].endswith("kparams"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+|_Z\S+):", l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith(".") or cur is None:
        continue
    cur[1].append(t.split(";")[0].strip())
tot = 0
for name, ins in blocks:
    ops = [i.split()[0] for i in ins]
    valu = sum(o.startswith("v_") for o in ops)
    f64 = sum(o.startswith("v_") and "_f64" in o for o in ops)
    mov = sum(o in ("v_mov_b64", "v_mov_b32", "v_cndmask_b32", "v_pk_mov_b32", "v_accvgpr_write_b32", "v_accvgpr_read_b32") for o in ops)
    salu = sum(o.startswith("s_") and not o.startswith("s_waitcnt") and not o.startswith("s_cbranch") and not o.startswith("s_branch") for o in ops)
    mem = sum(o.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_")) for o in ops)
    tot += len(ins)
    br = ops[-1] if ops and ("branch" in ops[-1]) else ""
    if len(ins) >= mn:
        print(f"{name:40s} n={len(ins):5d} valu={valu:5d} f64={f64:5d} mov/cnd={mov:4d} salu={salu:4d} mem={mem:3d} {br}")
    if dump and name == dump:
        print("\n".join(ins))
print("total instructions", tot)
