#!/usr/bin/env python3
"""Instruction mix of a kernel's outermost loop in /tmp/smj_kernels.s (run tools/kres.py first).

    python tools/isa_loop.py chunk_scatter_kernelILi2ELi10 [--dump]
"""
import re
import sys
from collections import Counter

s = open("/tmp/smj_kernels.s").read()
pat = sys.argv[1]
m = re.search(r"^(_Z\S*" + pat + r"\S*):", s, re.M)
a = m.start()
b = s.index(".Lfunc_end", a)
body = s[a:b].split("\n")
hdr = [i for i, l in enumerate(body) if "Loop Header: Depth=1" in l]
start = hdr[0] if hdr else 0
lab = body[start].split(":")[0]
ends = [i for i, l in enumerate(body) if lab in l and ("s_branch" in l or "s_cbranch" in l)]
end = max(ends) if ends else len(body) - 1
c = Counter()
for l in body[start:end + 1]:
    t = l.strip().split()
    if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
        continue
    op = t[0]
    if op.startswith("v_"):
        k = "valu"
    elif op.startswith("ds_"):
        k = "lds"
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        k = "vmem"
    elif op in ("s_waitcnt", "s_barrier"):
        k = op
    elif op.startswith("s_cbranch") or op == "s_branch":
        k = "branch"
    else:
        k = "salu"
    c[k] += 1
print(f"{m.group(1)[:80]}: loop lines {start}-{end}:", dict(c.most_common()))
if "--dump" in sys.argv:
    print("\n".join(body[start:end + 1]))
