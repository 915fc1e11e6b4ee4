"""Basic-block summary of one loop of an AMDGPU .s listing (diagnostic).

usage: python blocks.py file.s START_LINE END_LINE
Prints each block: label, instruction count (VALU/SALU/LDS/VMEM/branch/nop),
successors.  Used to count issue slots on a hot path by hand."""
import re, sys
f, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
lines = open(f).read().split("\n")[a - 1:b]
blocks = []
cur = None
for i, ln in enumerate(lines, a):
    m = re.match(r"^(\.LBB\w+):", ln) or re.match(r"^; %(bb\.\d+):", ln)
    if m:
        cur = {"label": m.group(1).replace("bb.", "%bb."), "line": i, "ins": [], "succ": []}
        blocks.append(cur)
        continue
    t = ln.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    if cur is None:
        cur = {"label": "start", "line": i, "ins": [], "succ": []}
        blocks.append(cur)
    op = t.split()[0]
    cur["ins"].append(op)
    if op.startswith("s_cbranch") or op == "s_branch":
        cur["succ"].append(t.split()[1])
def kind(op):
    if op.startswith("v_"): return "V"
    if op.startswith("s_nop"): return "N"
    if op.startswith("s_cbranch") or op == "s_branch": return "B"
    if op.startswith("s_waitcnt"): return "W"
    if op.startswith("s_"): return "S"
    if op.startswith("ds_"): return "L"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")): return "M"
    return "?"
for bl in blocks:
    c = {}
    for op in bl["ins"]:
        k = kind(op); c[k] = c.get(k, 0) + 1
    print("%-14s L%-7d n=%-3d %s -> %s" % (bl["label"], bl["line"], len(bl["ins"]),
          " ".join("%s%d" % (k, v) for k, v in sorted(c.items())), ",".join(bl["succ"])))
