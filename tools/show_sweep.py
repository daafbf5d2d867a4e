"""Print a sweep's bench lines: python tools/show_sweep.py TAG CFG"""
import glob
import json
import sys
tag, cfg = sys.argv[1], sys.argv[2]
leg = {}
for l in open(f"gpurun_out/{tag}_{cfg}_legend.txt").read().strip().split("\n"):
    k, _, v = l.partition(" ")
    leg[k] = v
for f in sorted(glob.glob(f"gpurun_out/{tag}_{cfg}_*.json"), key=lambda p: int(p.rsplit("_", 1)[1][:-5])):
    i = f.rsplit("_", 1)[1][:-5]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(i, leg.get(i, ""), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"],
              round(d["ms_per_step"] - d["roofline"]["kernel_ms"], 4))
    except Exception as e:
        print(i, leg.get(i, ""), "ERR", open(f).read()[-300:])
