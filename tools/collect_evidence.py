"""Copy a round's GPU evidence from gpurun_out/ (tools/gpu_evidence.sh ROUND) into profiles/ROUND/:
the default bench line, per-workload rocprofv3 kernel stats, the calibrated PMC traffic summary, the
MFMA counter pass, the C1 kernel stats and the tails of the GPU test logs.
usage: python tools/collect_evidence.py r05"""
import glob
import json
import os
import shutil
import sys

RD = sys.argv[1] if len(sys.argv) > 1 else "r05"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles", RD)
os.makedirs(P, exist_ok=True)
bench = os.path.join(G, f"{RD}_bench.log")
if os.path.exists(bench):
    line = [x for x in open(bench) if x.startswith("{")][-1]
    json.dump(json.loads(line), open(os.path.join(P, "bench_default.json"), "w"), indent=1)
for d in sorted(glob.glob(os.path.join(G, f"prof_{RD}", "*"))):
    key = os.path.basename(d)
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(P, f"{key}_kernel_stats.csv"))
    if key == "mfma":
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            shutil.copy(f, os.path.join(P, "c4_mfma_pmc.csv"))
tr = os.path.join(G, f"{RD}_traffic.json")
if os.path.exists(tr):
    shutil.copy(tr, os.path.join(P, "traffic.json"))
tails = []
for f in sorted(glob.glob(os.path.join(G, f"{RD}_test_*.log"))) + [os.path.join(G, f"{RD}_smoke.log")]:
    if os.path.exists(f):
        lines = open(f).read().strip().splitlines()
        tails.append(f"== {os.path.basename(f)}\n" + "\n".join(lines[-2:]))
if tails:
    open(os.path.join(P, "gpu_tests_tail.log"), "w").write("\n".join(tails) + "\n")
print("\n".join(sorted(os.listdir(P))))
