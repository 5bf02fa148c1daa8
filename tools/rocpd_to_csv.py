"""Convert a rocprofv3 SQLite output (*_results.db, the default format of this rocprofv3) into the CSV
files the other tools read: PREFIX_kernel_trace.csv (Kernel_Name, Start_Timestamp, End_Timestamp) and
PREFIX_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).
usage: python tools/rocpd_to_csv.py RESULTS.db OUT_PREFIX"""
import collections
import csv
import math
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
rows = [(names.get(k, str(k)), s, e) for k, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch")]
copies = []
try:
    copies = [("copy", s, e) for s, e in c.execute("select start, end from rocpd_memory_copy")]
except sqlite3.Error:
    pass
rows.sort(key=lambda r: r[1])
with open(out + "_kernel_trace.csv", "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    for r in rows:
        w.writerow(r)
agg = collections.defaultdict(list)
for n, s, e in rows:
    agg[n].append(e - s)
tot = sum(sum(v) for v in agg.values())
with open(out + "_kernel_stats.csv", "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
        w.writerow([n, len(v), sum(v), m, 100.0 * sum(v) / tot, min(v), max(v), sd])
print(f"{len(rows)} dispatches, {len(agg)} kernels, {len(copies)} memory copies -> {out}_kernel_*.csv")
