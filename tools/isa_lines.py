"""Static instruction mix per source line of one kernel (hipcc -gline-tables-only -S).

    python tools/isa_lines.py KERNEL_REGEX [N]
"""
import os
import re
import subprocess
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pim-sort-merge-join_amd")
out = "/tmp/smj_msd_g.s"
if not os.environ.get("NOBUILD"):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-gline-tables-only",
                           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
                           "--cuda-device-only", "-S", os.path.join(PKG, "csrc", "smj_msd.hip"), "-o", out],
                          stderr=subprocess.DEVNULL)
s = open(out).read()
m = re.search(r"^(_ZN3smj\S*" + sys.argv[1] + r"\S*):", s, re.M)
a = m.start()
b = s.index(".Lfunc_end", a)
files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
cur = None
per = defaultdict(Counter)
for l in s[a:b].split("\n"):
    t = l.strip()
    if t.startswith(".loc"):
        f = t.split()
        cur = (files.get(f[1], f[1]).split("/")[-1], int(f[2]))
        continue
    tt = t.split()
    if not tt or tt[0].startswith((".", ";")) or tt[0].endswith(":"):
        continue
    op = tt[0]
    k = ("valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else
         "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "salu")
    per[cur][k] += 1
rows = sorted(per.items(), key=lambda kv: -kv[1]["valu"])
print(m.group(1), "static valu", sum(c["valu"] for _, c in rows))
for k, c in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(k, dict(c))
