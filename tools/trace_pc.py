"""Average per-kernel durations of the last N calls in a per-call rocprofv3 kernel trace."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 6
calls = 40
agg = collections.defaultdict(list)
for r in rows[-per * calls:]:
    agg[r['Kernel_Name'][:80]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in agg.items():
    print(f"{k:80s} n={len(v)} avg {sum(v) / len(v):6.2f} us")
t0 = int(rows[-per * calls]['Start_Timestamp'])
t1 = int(rows[-1]['End_Timestamp'])
print('per call span (profiled)', round((t1 - t0) / 1000 / calls, 2))
