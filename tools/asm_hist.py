"""Diagnostic: per-basic-block instruction histogram of one kernel in a hipcc -S listing.
Usage: python tools/asm_hist.py file.s kernel_substring [--blocks]"""
import re
import sys
from collections import Counter

path, key = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
i0 = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l) and key in l.split(":")[0])
i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], ["entry", Counter(), []]
for l in lines[i0 + 1:i1]:
    t = l.strip()
    if re.match(r"^\.LBB\S*:", t):
        blocks.append(cur)
        cur = [t[:-1], Counter(), []]
        continue
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    cur[1][op] += 1
    if op.startswith("s_cbranch") or op == "s_branch":
        cur[2].append(t.split()[1])
blocks.append(cur)
order = {b[0]: n for n, b in enumerate(blocks)}
tot = Counter()
for b in blocks:
    tot.update(b[1])
print("total", sum(tot.values()))
for k, v in tot.most_common(40):
    print(f"{v:6d} {k}")
if "--blocks" in sys.argv:
    for n, (name, c, br) in enumerate(blocks):
        back = [x for x in br if x in order and order[x] <= n]
        ds = sum(v for k, v in c.items() if k.startswith("ds_"))
        f64 = sum(v for k, v in c.items() if k.endswith("f64") or "f64_" in k)
        print(f"{name:12s} n={sum(c.values()):5d} ds={ds:4d} f64={f64:4d} {'LOOP->' + ','.join(back) if back else ''}")
