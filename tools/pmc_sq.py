"""Summarise tools/pmc_sq.sh: per kernel, the SQ counters per launch (averaged over launches)."""
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    row = {c: v / max(n[(k, c)], 1) for c, v in d.items()}
    wc = row.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:24]:24s} waves {row.get('SQ_WAVES', 0):8.0f} wave_cyc {wc:10.0f}  wait {row.get('SQ_WAIT_ANY', 0) / wc:5.2f}"
          f"  stall {row.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f}  active {row.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}"
          f"  valu {row.get('SQ_INSTS_VALU', 0):9.0f} lds {row.get('SQ_INSTS_LDS', 0):8.0f} busy {row.get('SQ_BUSY_CYCLES', 0):8.0f}")
