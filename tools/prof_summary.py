"""Summarise a rocprofv3 --kernel-trace database (run_results.db) into
  <out>_stats.csv   per-kernel Calls/Total/Average/Min/Max (rocprofv3 --stats layout)
  <out>_by_grid.txt per-kernel, per-grid-size medians (the timed launches of
                    bench.py are the ones at the half-ensemble grid size)
plus the resource line (VGPR/SGPR/LDS/scratch) of each kernel.

  python tools/prof_summary.py gpurun_out/prof_v4/run_results.db profiles/r01/bench_v4
"""
import sqlite3
import statistics
import sys
from collections import defaultdict


def _short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0]


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, "
                     "sgpr_count, lds_size, scratch_size from kernels").fetchall()
    by = defaultdict(list)
    grid = defaultdict(list)
    res = {}
    for name, dur, gx, wx, v, av, s, lds, scr in rows:
        by[name].append(dur)
        grid[(name, gx)].append(dur)
        res[name] = (wx, v, av, s, lds, scr)
    total = sum(sum(d) for d in by.values())
    with open(out + "_stats.csv", "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n')
        for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            sd = statistics.pstdev(d) if len(d) > 1 else 0.0
            f.write('"%s",%d,%d,%f,%.2f,%d,%d,%f\n' % (name, len(d), sum(d), sum(d) / len(d),
                                                      100.0 * sum(d) / total, min(d), max(d), sd))
    with open(out + "_by_grid.txt", "w") as f:
        for (name, gx), d in sorted(grid.items()):
            short = _short(name)
            f.write("%-28s grid %8d launches %4d median %7.1f us mean %7.1f us\n"
                    % (short[:28], gx, len(d), statistics.median(d) / 1e3, sum(d) / len(d) / 1e3))
        f.write("\n# resources: workgroup, arch VGPR, accum VGPR, SGPR, LDS bytes, scratch bytes\n")
        for name, r in sorted(res.items()):
            short = _short(name)
            f.write("%-28s wg %4d vgpr %3d agpr %3d sgpr %3d lds %6d scratch %5d\n" % ((short[:28],) + r))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
