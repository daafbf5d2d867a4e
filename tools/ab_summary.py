"""Summarise tools/ab.sh output: python tools/ab_summary.py TAG"""
import glob, json, os, sys
tag = sys.argv[1]
rows = {}
for f in sorted(glob.glob(f"gpurun_out/{tag}_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unparsable", e); continue
    print(f"{os.path.basename(f):28s} value {d['value']:12.1f}  ms/step {d['ms_per_step']:.4f}  kernel_ms {d['roofline']['kernel_ms']:.4f}  frac {d['roofline']['frac']:.4f}")
