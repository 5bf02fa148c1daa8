"""Compare rocprofv3 kernel-stats CSVs side by side: average us per launch and launches.
usage: python tools/kcmp.py a_kernel_stats.csv [b_kernel_stats.csv ...] [--per N]  (N = steps, to print us per step)"""
import csv
import re
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"]
        m = re.search(r"(k_[A-Za-z0-9_]+(?:<[^>]*>)?)", n)
        k = m.group(1) if m else n[:40]
        a = out.setdefault(k, [0, 0.0])
        a[0] += int(r["Calls"]); a[1] += float(r["TotalDurationNs"])
    return out


args = [a for a in sys.argv[1:] if not a.startswith("--")]
per = None
if "--per" in sys.argv:
    per = float(sys.argv[sys.argv.index("--per") + 1])
    args = [a for a in args if a != sys.argv[sys.argv.index("--per") + 1]]
tabs = [load(a) for a in args]
keys = sorted(set().union(*tabs), key=lambda k: -max(t.get(k, [0, 0])[1] for t in tabs))
for k in keys:
    cells = []
    for t in tabs:
        c, ns = t.get(k, [0, 0.0])
        cells.append(f"{c:6d} {ns / max(c, 1) / 1e3:7.1f}" + (f" {ns / 1e3 / per:7.1f}" if per else ""))
    print(f"{k[:44]:44s} " + " | ".join(cells))
tot = [sum(v[1] for v in t.values()) for t in tabs]
print("total ms", " | ".join(f"{x / 1e6:.3f}" for x in tot))
