"""Attribute a kernel's instructions to source lines (.loc) in a hipcc -S -gline-tables-only
listing.  usage: isa_by_line.py file.s mangled-substring [top]"""
import collections
import re
import sys

src, key = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(src).read().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]+)"(?:\s+"([^"]+)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur = "?"
cnt = collections.Counter()
kinds = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    t = l.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    k = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else "m"
    cnt[cur] += 1
    kinds[cur][k] += 1
for loc, n in cnt.most_common(top):
    print(f"{n:5d}  v{kinds[loc]['v']:4d} s{kinds[loc]['s']:4d} ds{kinds[loc]['ds']:3d} m{kinds[loc]['m']:3d}  {loc}")
