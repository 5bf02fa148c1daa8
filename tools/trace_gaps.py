"""Timeline of a rocprofv3 kernel trace: per step of the chained LocalMapping step (delimited by a
marker kernel), the device-busy time, the idle gaps before each launch, and the largest gaps by the
kernel that follows them.  usage: python tools/trace_gaps.py KERNEL_TRACE.csv [step_marker_kernel]"""
import collections
import csv
import sys


def short(n):
    name = n.split('::')[1].split('(')[0] if '::' in n else n.split('(')[0][:40]
    for tag in ('<true>', '<false>', '<0>', '<1>'):
        if tag in n and tag not in name:
            name += tag
    return name


rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "k_bf_scan"
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
# steps: from one marker launch to the next
idx = [i for i, e in enumerate(ev) if e[2].startswith(marker)]
steps = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1)]
if not steps:
    sys.exit("no steps found")
gap_by = collections.defaultdict(list)
dur_by = collections.defaultdict(list)
spans, busy = [], []
for a, b in steps[2:]:  # skip warm-up steps
    spans.append(ev[b][0] - ev[a][0])
    bz = 0
    for i in range(a, b):
        s, e, n = ev[i]
        dur_by[n].append(e - s)
        bz += e - s
        if i > a:
            gap_by[n].append(max(0, s - ev[i - 1][1]))
    busy.append(bz)
ns = len(spans)
print(f"steps {ns}: span {sum(spans) / ns / 1e3:.1f} us, kernels busy {sum(busy) / ns / 1e3:.1f} us, "
      f"idle {(sum(spans) - sum(busy)) / ns / 1e3:.1f} us per step")
print(f"{'kernel':44s} {'per_step':>8s} {'avg_us':>8s} {'gap_before_us(avg)':>18s} {'gap_per_step':>12s}")
for n in sorted(dur_by, key=lambda k: -sum(dur_by[k])):
    d, g = dur_by[n], gap_by.get(n, [0])
    print(f"{n[:44]:44s} {len(d) / ns:8.1f} {sum(d) / len(d) / 1e3:8.2f} {sum(g) / max(len(g), 1) / 1e3:18.2f} "
          f"{sum(g) / ns / 1e3:12.2f}")
