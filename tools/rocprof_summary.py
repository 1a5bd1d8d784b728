"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite .db or kernel_stats/kernel_trace CSV) into
a per-kernel table: calls, total/avg/min/max duration (us), VGPR/AGPR/SGPR, scratch bytes per lane.

usage: python tools/rocprof_summary.py <run_results.db | kernel_trace.csv> [> profiles/rNN_*.txt]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0]


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, duration, vgpr_count, accum_vgpr_count, sgpr_count, scratch_size, grid_x, workgroup_x "
         "from kernels")
    for r in c.execute(q):
        yield {"name": r[0], "ns": float(r[1]), "vgpr": r[2], "agpr": r[3], "sgpr": r[4], "scratch": r[5],
               "grid": r[6], "wg": r[7]}


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield {"name": r["Kernel_Name"], "ns": float(r["End_Timestamp"]) - float(r["Start_Timestamp"]),
                   "vgpr": r.get("VGPR_Count"), "agpr": r.get("Accum_VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                   "scratch": r.get("Scratch_Size"), "grid": r.get("Grid_Size"), "wg": r.get("Workgroup_Size")}


def main(path):
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    agg = defaultdict(list)
    meta = {}
    for r in rows:
        k = short(r["name"])
        agg[k].append(r["ns"])
        meta[k] = r
    # rocpd stores durations in ns
    tot = sum(sum(v) for v in agg.values())
    print("%-28s %6s %12s %12s %12s %12s %6s  %s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us",
                                                   "pct", "vgpr/agpr/sgpr scratch grid wg"))
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        m = meta[k]
        print("%-28s %6d %12.1f %12.1f %12.1f %12.1f %6.2f  %s/%s/%s %s %s %s" % (
            k[-28:], len(v), sum(v) / 1e3, sum(v) / len(v) / 1e3, min(v) / 1e3, max(v) / 1e3, 100 * sum(v) / tot,
            m["vgpr"], m["agpr"], m["sgpr"], m["scratch"], m["grid"], m["wg"]))


if __name__ == "__main__":
    main(sys.argv[1])
