"""Summarise a rocprofv3 --kernel-trace csv of tools/chain_drift.py: per
kernel (name, grid) the duration percentiles in consecutive windows of the
run, to see which kernel slows down as the chain moves.

  python tools/drift_trace.py gpurun_out/<dir>/run_kernel_trace.csv [windows=8]
"""
import collections
import csv
import sys

import numpy as np

rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if not n.startswith("k_"):
        continue
    rows[(n, int(r["Grid_Size_X"]))].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
nw = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for k, v in sorted(rows.items()):
    if len(v) < 100:
        continue
    v.sort()
    d = np.array([x[1] for x in v]) / 1e3
    print("%-22s grid %7d n %6d" % (k[0], k[1], len(d)))
    for i, c in enumerate(np.array_split(d, nw)):
        print("   window %d: median %7.1f  p90 %7.1f  p99 %8.1f  max %8.1f us" % (
            i, np.median(c), np.percentile(c, 90), np.percentile(c, 99), c.max()))
