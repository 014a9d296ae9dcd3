"""HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_profile.sh, for bench.py's roofline.traffic.

  python tools/pmc_traffic.py gpurun_out/pmc_<tag> profiles/r03/pmc_traffic_c2.json [pairs [npts nsub [grid]]]

pairs = (walker, eclipse) pairs per launch of the profiled run (bench.py
defaults: 512 = 1024 walkers / 2 halves x 1 eclipse); bench.py scales by it.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
  * rocprofv3 reports FETCH_SIZE and WRITE_SIZE in KiB;
  * on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced read, so
    it is doubled; WRITE_SIZE is taken as is.
SQ_INSTS_VALU_FLOPS_FP64 (ADD + MUL + TRANS + 2 FMA, per wave instruction)
times 64 lanes gives the executed FP64 FLOPs.
Only dispatches of the bench's timed size (the most common grid size of each
kernel) are kept, and the median per dispatch is reported.  The counters see
memory-side fabric requests (Infinity-Cache hits included), so the figure is
an upper bound on HBM bytes.
"""
import collections
import csv
import glob
import json
import os
import sys

FETCH_CORR = 2.0
KIB = 1024.0


def per_dispatch(d, counter):
    """{kernel: [(grid, value), ...]} of one counter over every pass under d."""
    out = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        grid = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            kn = kn.split("(")[0]
            key = (r["Dispatch_Id"], kn)
            per[key] += float(r["Counter_Value"])
            grid[key] = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        for key, v in per.items():
            out[key[1]].append((grid[key], v))
    return out


def summarise(d, grid=None):
    fetch = per_dispatch(d, "FETCH_SIZE")
    write = per_dispatch(d, "WRITE_SIZE")
    flops = per_dispatch(d, "SQ_INSTS_VALU_FLOPS_FP64")  # per wave instruction: x64 lanes
    res = {}
    for kn in sorted(set(fetch) | set(write)):
        if not kn.startswith("k_"):
            continue
        row = {}
        for name, src, corr in (("fetch_bytes", fetch, FETCH_CORR), ("write_bytes", write, 1.0),
                                ("fp64_flops", flops, 64.0 / KIB)):
            vals = src.get(kn, [])
            if not vals:
                continue
            g = grid if grid and any(gs == grid for gs, _ in vals) else \
                collections.Counter(gs for gs, _ in vals).most_common(1)[0][0]
            sel = sorted(v for gs, v in vals if gs == g)
            row[name] = sel[len(sel) // 2] * KIB * corr
            row["grid"] = g
            row[name + "_dispatches"] = len(sel)
        if "fetch_bytes" in row and "write_bytes" in row:
            row["traffic_bytes"] = row["fetch_bytes"] + row["write_bytes"]
        res[kn] = row
    return res


if __name__ == "__main__":
    src, dst = sys.argv[1], sys.argv[2]
    pairs = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    # optional 6th argument: the grid size of the timed launches (when as many
    # other launches of the kernel ran, e.g. initialise_walkers' larger batch)
    res = summarise(src, int(sys.argv[6]) if len(sys.argv) > 6 else None)
    meta = {"source": os.path.basename(os.path.normpath(src)), "pairs_per_launch": pairs,
            "npts": int(sys.argv[4]) if len(sys.argv) > 4 else 300,
            "nsub": int(sys.argv[5]) if len(sys.argv) > 5 else 1,
            "note": "median per dispatch of the bench's timed launches; FETCH_SIZE x2 (gfx950); KiB -> bytes"}
    with open(dst, "w") as fh:
        json.dump({"meta": meta, "kernels": res}, fh, indent=1)
    for k, v in res.items():
        print(k, {a: (round(b) if isinstance(b, float) else b) for a, b in v.items()})
