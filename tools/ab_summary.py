"""Summarise a tools/session.sh `ab` step: python tools/ab_summary.py <gpurun_out> <TAG>
Per value of the A/B knob: every run's ms/step and dominant-kernel ms, then the mean."""
import glob
import json
import os
import re
import sys
from collections import defaultdict

out, tag = sys.argv[1], sys.argv[2]
agg = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, f"{tag}_ab_*_*.json"))):
    m = re.match(rf"{re.escape(tag)}_ab_(.+)_(\d+)\.json$", os.path.basename(f))
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError) as e:
        print(f, "unparsable", e)
        continue
    agg[m.group(1)].append((d["ms_per_step"], d["roofline"]["kernel_ms"]))
    print(f"{os.path.basename(f):36s} value {d['value']:12.1f}  ms/step {d['ms_per_step']:.4f}  "
          f"kernel_ms {d['roofline']['kernel_ms']:.4f}  frac {d['roofline']['frac']:.4f}")
for v, xs in agg.items():
    print(f"{v:>12s}: ms/step mean {sum(a for a, _ in xs) / len(xs):.4f}  kernel_ms mean {sum(b for _, b in xs) / len(xs):.4f}"
          f"  ({len(xs)} runs)")
