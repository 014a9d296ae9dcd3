"""Summarise rocprofv3 --pmc passes (tools/pmc_profile.sh) per kernel: mean
counter value per dispatch of the bench's timed-size launches."""
import csv, collections, glob, os, sys
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*/run_counter_collection.csv"))):
    per = collections.defaultdict(float)
    key = {}
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = (r["Dispatch_Id"], kn.split("(")[0].split("<")[0], r["Counter_Name"])
        per[k] += float(r["Counter_Value"])
        key[k] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    for (disp, kern, cn), v in per.items():
        acc[kern][cn].append(v)
for kern, cs in acc.items():
    if not kern.startswith("k_"):
        continue
    print(kern)
    for cn, vals in sorted(cs.items()):
        vals = sorted(vals)
        print("   %-28s median %.4g  (n=%d)" % (cn, vals[len(vals) // 2], len(vals)))
