"""Static instruction mix of a kernel's outermost step loop in a hipcc -S listing.
usage: isa_loop_stats.py file.s mangled-substring"""
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and key in l.split(":")[0]))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
# outermost loop = the first "Loop Header: Depth=1" label that encloses the most lines
hdrs = [i for i, l in enumerate(body) if "Loop Header" in l and "Depth=1" in l]
best = None
for h in hdrs:
    lab = body[h].split(":")[0]
    last = max((j for j, l in enumerate(body) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", l)),
               default=h)
    # blocks 'in Loop: Header=BBx' after the back-edge belong to the loop too
    tag = "Header=" + lab.replace(".LBB", "BB")
    last = max([last] + [j for j, l in enumerate(body) if tag in l])
    while last + 1 < len(body) and not body[last + 1].startswith(".LBB"):
        last += 1
    if best is None or last - h > best[1] - best[0]:
        best = (h, last)
h, last = best
# loop preheader-jump form: blocks labelled 'in Loop: Header=...' before the header
tag = "Header=" + body[h].split(":")[0].replace(".LBB", "BB")
first = min([h] + [j for j, l in enumerate(body) if tag in l])
cnt = {"valu": 0, "salu": 0, "ds": 0, "vmem": 0, "barrier": 0, "branch": 0}
ops = {}
for l in body[first:last + 1]:
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    ops[op] = ops.get(op, 0) + 1
    if op.startswith("v_"):
        cnt["valu"] += 1
    elif op.startswith("ds_"):
        cnt["ds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cnt["vmem"] += 1
    elif op == "s_barrier":
        cnt["barrier"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        cnt["branch"] += 1
    elif op.startswith("s_"):
        cnt["salu"] += 1
print(cnt)
if len(sys.argv) > 3:
    for op, n in sorted(ops.items(), key=lambda x: -x[1])[:40]:
        print(f"{n:5d} {op}")
