#!/usr/bin/env python3
"""Per-kernel resources (LDS, VGPRs, scratch, spills) of the gfx950 build.

    python tools/kres.py [regex]      # compiles csrc/smj_kernels.hip to /tmp/smj_kernels.s
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pim-sort-merge-join_amd")
out = "/tmp/smj_kernels.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
                       "--cuda-device-only", "-S", os.path.join(PKG, "csrc", "smj_kernels.hip"), "-o", out],
                      stderr=subprocess.DEVNULL)
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
s = open(out).read()
md = s[s.index("amdhsa.kernels:"):]
for b in re.split(r"\n  - ", md):
    m = re.search(r"\.name:\s+(\S+)", b)
    if not m or not pat.search(m.group(1)):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", b) or [None, None])[1]
    print(f"{m.group(1)[:72]:72s} lds={g('group_segment_fixed_size')} vgpr={g('vgpr_count')} "
          f"scratch={g('private_segment_fixed_size')} spill={g('vgpr_spill_count')}")
