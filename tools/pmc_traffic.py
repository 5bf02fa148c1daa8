"""Reduce rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in SEPARATE runs) to HBM
bytes per launch per kernel, and the --stats kernel summary to average durations.

    python tools/pmc_traffic.py PROF_DIR OUT_JSON [--workload KEY]

With --workload the summary is merged into OUT_JSON under "workloads": {KEY: ...} (the layout
bench.py reads), so one file holds every profiled workload.

PROF_DIR holds the rocprofv3 CSV outputs (searched recursively): *counter_collection.csv from
the FETCH_SIZE and WRITE_SIZE passes and *kernel_stats.csv from the --kernel-trace --stats pass.
Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950
FETCH_SIZE tallies 128-B fabric read requests of wide coalesced streaming reads at 64 B; the
calibration of tools/micro/fetch_cal.hip (profiles/r04/fetch_calibration.json: every byte of a
96 MiB buffer read once per pattern, caches evicted in between) measured, FETCH_SIZE / unique bytes:
16 B and 8 B per lane consecutive 0.50; a 96-byte record per lane at random slots 1.00; a 48-byte
record per lane at random slots 1.67 (lines shared by two records fetched twice); one 8-byte read per
random 64-byte line 1.00 (of the lines' bytes).  So the x2 correction holds for streaming kernels
only: kernels whose reads are record gathers by index (GATHER below) are taken at x1.  WRITE_SIZE
reads the bytes exactly for 16-B streaming stores and for 96-byte records at random slots (1.01);
48-byte records at random slots 1.35 (partial lines).
"""
import csv
import glob
import json
import os
import re
import sys

SHORT = re.compile(r"(k_[a-z0-9_]+)")
# kernels whose reads are dominated by record gathers by index (FETCH_SIZE x1, see above)
GATHER = {"k_ba_schur", "k_ba_backsub", "k_db_gather", "k_db_pairs", "k_db_place", "k_db_result",
          "k_db_result64", "k_db_segsort", "k_resolve", "k_cand_frame", "k_cand_local"}


def fetch_factor(kernel):
    return 1.0 if kernel in GATHER else 2.0


def short_name(name):
    m = SHORT.search(name)
    return m.group(1) if m else name


def main(prof_dir, out, workload=None):
    per = {}
    for path in glob.glob(os.path.join(prof_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                ctr = row.get("Counter_Name", "")
                if ctr not in ("FETCH_SIZE", "WRITE_SIZE"):
                    continue
                k = short_name(row.get("Kernel_Name", ""))
                v = float(row.get("Counter_Value", 0.0)) * 1024.0
                if ctr == "FETCH_SIZE":
                    v *= fetch_factor(k)  # gfx950 correction (streaming x2, gathers x1)
                d = per.setdefault(k, {}).setdefault(ctr, {})
                disp = row.get("Dispatch_Id", str(len(d)))
                d[disp] = d.get(disp, 0.0) + v  # counters are summed over dimensions / XCDs
    stats = {}
    for path in glob.glob(os.path.join(prof_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short_name(row.get("Name", ""))
                s = stats.setdefault(k, {"calls": 0, "total_ns": 0.0})
                s["calls"] += int(row.get("Calls", 0))
                s["total_ns"] += float(row.get("TotalDurationNs", 0.0))
    kernels = {}
    for k in sorted(set(per) | set(stats)):
        e = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            vals = list(per.get(k, {}).get(ctr, {}).values())
            if vals:
                e[ctr.lower() + "_bytes_per_launch"] = sum(vals) / len(vals)
        if "fetch_size_bytes_per_launch" in e and "write_size_bytes_per_launch" in e:
            e["hbm_bytes_per_launch"] = e["fetch_size_bytes_per_launch"] + e["write_size_bytes_per_launch"]
        if k in stats and stats[k]["calls"]:
            e["calls"] = stats[k]["calls"]
            e["avg_us"] = stats[k]["total_ns"] / stats[k]["calls"] / 1e3
        kernels[k] = e
    for k, e in kernels.items():
        e["fetch_correction"] = fetch_factor(k)
    summary = {"source": prof_dir, "fetch_correction": "x2 streaming, x1 gather kernels (tools/pmc_traffic.py GATHER)",
               "kernels": kernels}
    if workload:
        try:
            with open(out) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            doc = {}
        doc.setdefault("workloads", {})[workload] = summary
    else:
        doc = summary
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k, e in kernels.items():
        print(k, e)


if __name__ == "__main__":
    args = sys.argv[1:]
    wl = None
    if "--workload" in args:
        i = args.index("--workload")
        wl = args[i + 1]
        del args[i:i + 2]
    main(args[0], args[1], wl)
