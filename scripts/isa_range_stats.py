"""Instruction mix of a line range of an asm listing: isa_range_stats.py file.s first last"""
import sys
lines = open(sys.argv[1]).read().split("\n")[int(sys.argv[2]) - 1:int(sys.argv[3])]
cnt = {"valu": 0, "salu": 0, "ds": 0, "vmem": 0, "barrier": 0, "branch": 0, "readlane": 0, "nop": 0}
for l in lines:
    t = l.strip()
    if not t or t.startswith((";", ".")):
        continue
    op = t.split()[0]
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        cnt["readlane"] += 1
    if op.startswith("v_"):
        cnt["valu"] += 1
    elif op.startswith("ds_"):
        cnt["ds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cnt["vmem"] += 1
    elif op == "s_barrier":
        cnt["barrier"] += 1
    elif op.startswith(("s_cbranch", "s_branch")):
        cnt["branch"] += 1
    elif op == "s_nop":
        cnt["nop"] += 1
    elif op.startswith("s_"):
        cnt["salu"] += 1
print(cnt)
