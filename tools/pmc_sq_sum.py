"""Summarise tools/pmc_sq.sh passes: per kernel, counters summed over its
dispatches, per wave and relative to SQ_WAVE_CYCLES.

    python tools/pmc_sq_sum.py gpurun_out/TAG
"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(root, "sq*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if c.get("SQ_WAVE_CYCLES", 0) < 1e6:
        continue
    waves = max(c.get("SQ_WAVES", 1.0), 1.0)
    per_wave = {n[3:]: round(v / waves) for n, v in sorted(c.items()) if n.startswith("SQ_INSTS")}
    frac = {n[3:]: round(v / c["SQ_WAVE_CYCLES"], 3) for n, v in sorted(c.items())
            if n.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
    print(f"{k[:48]:48s} waves={int(waves)} insts/wave={per_wave} cycles-frac={frac}")
