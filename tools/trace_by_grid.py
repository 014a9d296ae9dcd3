"""Per (kernel, grid size) median/min/max durations of a rocprofv3
--kernel-trace csv (run_kernel_trace.csv), in us.
  python tools/trace_by_grid.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

import numpy as np

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if n.startswith("k_"):
        d[(n, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v = np.array(v)
    print("%-26s grid %9d launches %4d median %8.1f min %8.1f max %8.1f" % (k[0], k[1], len(v), np.median(v),
                                                                             v.min(), v.max()))
