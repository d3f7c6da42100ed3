"""Attribute a kernel's instructions to the train-body line they are inlined
into (the outermost rl_train_impl.h call site below the kernel wrapper), in a
hipcc -S -gline-tables-only listing.
usage: isa_by_callsite.py file.s mangled-substring first_line last_line [top]"""
import collections
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lo, hi = int(sys.argv[3]), int(sys.argv[4])
top = int(sys.argv[5]) if len(sys.argv) > 5 else 40
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur = None
cnt = collections.Counter()
kinds = collections.defaultdict(collections.Counter)
for l in lines[start:end]:
    t = l.strip()
    if t.startswith(".loc"):
        body = [int(m) for m in re.findall(r"rl_train_impl\.h:(\d+)", t)]
        body = [b for b in body if lo <= b <= hi]
        cur = body[-1] if body else None
        continue
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    if cur is None:
        continue
    op = t.split()[0]
    k = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else "m"
    cnt[cur] += 1
    kinds[cur][k] += 1
tot = collections.Counter()
for ln, n in cnt.most_common(top):
    print(f"{n:5d}  v{kinds[ln]['v']:4d} s{kinds[ln]['s']:4d} ds{kinds[ln]['ds']:3d} m{kinds[ln]['m']:3d}  line {ln}")
for ln in cnt:
    for k, v in kinds[ln].items():
        tot[k] += v
print("total", dict(tot))
