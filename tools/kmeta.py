"""Per-kernel resource metadata (VGPRs, SGPRs, spills, LDS) of a hipcc -S listing.

    python tools/kmeta.py /tmp/msd.s REGEX...
"""
import re
import sys

s = open(sys.argv[1]).read()
meta = s[s.index("amdhsa.kernels:"):]
for ent in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", ent)
    if not name or not any(re.search(p, name.group(1)) for p in sys.argv[2:]):
        continue
    f = dict(re.findall(r"\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size|private_segment_fixed_size):\s+(\d+)", ent))
    print(name.group(1)[:60], f)
