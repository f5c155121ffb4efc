"""Prints the group loop (the loop whose header holds the first ds_read_b128)
of the n-th kernel whose symbol contains `pattern` in an ISA listing, plus
the kernel's register counts: python scripts/isa_loop.py <file.s> <pattern> [n] [extra lines]"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
pat, nth = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0
extra = int(sys.argv[4]) if len(sys.argv) > 4 else 0
k = -1
for s, l in enumerate(lines):
    if re.match(r"^_Z\w+:", l) and pat in l:
        k += 1
        if k == nth:
            break
else:
    sys.exit("no such kernel")
e = s
while not lines[e].startswith(".Lfunc_end"):
    e += 1
seg = lines[s:e]
first = next(i for i, x in enumerate(seg) if "ds_read_b128" in x)
hdr = max(i for i in range(first) if re.match(r"^\.LBB\d+_\d+:", seg[i]))
lab = seg[hdr].split(":")[0]
back = max(i for i, x in enumerate(seg) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", x))
print(l.split(":")[0])
for x in seg[hdr:back + 1 + extra]:
    x = x.split(";")[0].rstrip()
    if x.strip():
        print(x)
meta = "\n".join(lines[e:e + 200000])
m = re.search(re.escape(l.split(":")[0]) + r"[\s\S]*?\.vgpr_count:\s+(\d+)[\s\S]*?\.vgpr_spill_count:\s+(\d+)", meta)
if m:
    print("vgpr_count", m.group(1), "spill", m.group(2))
