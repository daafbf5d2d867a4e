"""Average PMC counters per dispatch for kernels matching a substring: python tools/pmc_summary.py TAG substr"""
import collections, csv, glob, sys
tag, sub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for d in sorted(glob.glob(f"gpurun_out/{tag}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(d)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(agg.get("SQ_WAVES", [1])) / max(len(agg.get("SQ_WAVES", [1])), 1)
for c, v in sorted(agg.items()):
    m = sum(v) / len(v)
    print(f"{c:30s} {m:16.1f}   per-wave {m / waves:12.2f}")
