"""Scratch spill sites (source lines) of one kernel: python tools/spills.py KERNEL_REGEX"""
import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pim-sort-merge-join_amd")
out = "/tmp/smj_msd_g.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-gline-tables-only",
                       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"), "--cuda-device-only",
                       "-S", os.path.join(PKG, "csrc", "smj_msd.hip"), "-o", out] + sys.argv[2:], stderr=subprocess.DEVNULL)
s = open(out).read()
m = re.search(r"^(_ZN3smj\S*" + sys.argv[1] + r"\S*):", s, re.M)
a = m.start()
b = s.index(".Lfunc_end", a)
files = dict(re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s))
cur = None
c = Counter()
for l in s[a:b].split("\n"):
    t = l.strip()
    if t.startswith(".loc"):
        f = t.split()
        cur = (files.get(f[1], f[1]).split("/")[-1], int(f[2]))
        continue
    if "scratch_" in t:
        c[(cur, t.split()[0])] += 1
for k, v in sorted(c.items()):
    print(k, v)
