"""For each render_mfma_k5r kernel in an ISA listing: the group loop (the loop
whose header holds the first ds_read_b128 of the record operands), its length
and the scratch (spill) instructions inside it, plus the kernel's totals."""
import re
import sys

lines = open(sys.argv[1] if len(sys.argv) > 1 else "raytracing2-fork_amd/build/rt2_render.s").read().split("\n")
pat = sys.argv[2] if len(sys.argv) > 2 else "render_mfma_k5r"
for s, l in enumerate(lines):
    if not (re.match(r"^_Z\w+:", l) and pat in l):
        continue
    e = s
    while not lines[e].startswith(".Lfunc_end"):
        e += 1
    seg = lines[s:e]
    first = next((i for i, x in enumerate(seg) if "ds_read_b128" in x), None)
    if first is None:
        continue
    hdr = max(i for i in range(first) if re.match(r"^\.LBB\d+_\d+:", seg[i]))
    lab = seg[hdr].split(":")[0]
    back = max(i for i, x in enumerate(seg) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", x))
    body = seg[hdr:back + 1]
    spills = [x.strip() for x in body if "scratch_" in x]
    vg = re.search(r"\.vgpr_count:\s+(\d+)", "\n".join(lines[e:e + 4000]))
    print(l.split(":")[0][-70:], f"loop {hdr}-{back} ({len(body)} lines), scratch in loop {len(spills)}, "
          f"kernel scratch ops {sum('scratch_' in x for x in seg)}")
