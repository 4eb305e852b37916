"""Per-dispatch averages of gpurun_out/pmcx/p*/ counters for the sweep kernels,
normalised per config (R=64 n=7 sweep unless CONFIGS is set)."""
import collections
import csv
import glob
import os

CFG = float(os.environ.get("CONFIGS", 621216192))
for f in sorted(glob.glob("gpurun_out/pmcx/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "sweep" not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(disp[k])
        print(f, k[:45])
        for c, x in sorted(v.items()):
            print(f"   {c:28s} {x / n:14.4g}   per config-lane {x / n / (CFG / 64):10.2f}")
