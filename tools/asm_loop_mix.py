#!/usr/bin/env python3
"""Instruction mix of a kernel's loops in hipcc's gfx950 assembly (dev tool).

usage: tools/asm_loop_mix.py file.s KERNEL_SUBSTRING [HEADER_LABEL]
Without HEADER_LABEL: lists the loop headers (from hipcc's "in Loop: Header=" comments) with
their instruction counts.  With it: the mix of that loop's blocks and its v_readlane /
v_writelane lines (SGPR spill traffic)."""
import collections
import re
import sys

src, kname = sys.argv[1], sys.argv[2]
hdr = sys.argv[3] if len(sys.argv) > 3 else None
s = open(src).read()
m = re.search(r"^(\w*" + re.escape(kname) + r"\w*):", s, flags=re.M)
if not m:
    sys.exit(f"kernel {kname} not found")
body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
loops = collections.defaultdict(list)
cur = []
for ln in body:
    if ln.startswith(".LBB") or ln.startswith("; %bb."):
        cur = re.findall(r"Header=(BB\d+_\d+)", ln)
        lab = ln.split(":")[0].lstrip(".") if ln.startswith(".LBB") else None
        if lab and lab[1:] not in cur:
            pass
    t = ln.strip().split()
    if cur and t and not t[0].startswith((".", ";")):
        loops[cur[0]].append(ln.strip())
if hdr is None:
    for h, ins in sorted(loops.items(), key=lambda kv: -len(kv[1])):
        c = collections.Counter(i.split()[0] for i in ins)
        print(f"{h}: {len(ins)} instructions, v_readlane {c['v_readlane_b32']}, v_writelane {c['v_writelane_b32']}, "
              f"f64 fma/mul/add {c['v_fma_f64'] + c['v_fmac_f64_e32']}/{c['v_mul_f64']}/{c['v_add_f64']}")
else:
    ins = loops[hdr]
    c = collections.Counter(i.split()[0] for i in ins)
    print(len(ins), c.most_common(40))
    for i in ins:
        if "lane_b32" in i:
            print("  ", i)
