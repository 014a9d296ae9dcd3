"""Summarise rocprofv3 --pmc passes (tools/pmc_profile.sh) per kernel: the
median counter value per dispatch over the dispatches of each kernel's most
common grid size (the bench's timed launches).

  python tools/pmc_summary.py gpurun_out/pmc_<tag>
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        k = (r["Dispatch_Id"], kn, r["Counter_Name"])
        per[k] += float(r["Counter_Value"])
        grid[k] = r.get("Grid_Size") or r.get("Grid_Size_X")
    for (disp, kern, cn), v in per.items():
        acc[kern][(grid[(disp, kern, cn)], cn)].append(v)
for kern in sorted(acc):
    if not kern.startswith("k_"):
        continue
    cs = acc[kern]
    g = collections.Counter(gs for (gs, _), vals in cs.items() for _ in vals).most_common(1)[0][0]
    print("%s  (grid %s)" % (kern, g))
    for (gs, cn), vals in sorted(cs.items(), key=lambda t: t[0][1]):
        if gs != g:
            continue
        vals = sorted(vals)
        print("   %-28s median %.4g  (n=%d)" % (cn, vals[len(vals) // 2], len(vals)))
