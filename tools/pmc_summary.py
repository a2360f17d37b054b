"""Summarise rocprofv3 PMC csvs (gpurun_out/pmc*/k_counter_collection.csv) for one kernel name pattern."""
import collections, csv, glob, sys
pat = sys.argv[1] if len(sys.argv) > 1 else "stage_kernel"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/k_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:36s} n={len(v):4d} mean={sum(v)/len(v):14.1f}")
