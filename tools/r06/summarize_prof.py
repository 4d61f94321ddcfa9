"""Reduce rocprofv3 output dirs (kernel stats, PMC counter collections) to
small text summaries so gpurun_out stays under its size cap.
usage: summarize_prof.py OUT.txt DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = open(sys.argv[1], "w")
for d in sys.argv[2:]:
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        out.write(f"== {f}\n")
        rows = list(csv.DictReader(open(f)))
        for r in rows[:25]:
            out.write(f"{r.get('Name','')[:90]:90s} calls {r.get('Calls')} avg_ns {r.get('AverageNs')} "
                      f"total_ns {r.get('TotalDurationNs')}\n")
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        out.write(f"== {f}\n")
        agg = defaultdict(lambda: defaultdict(float))
        cnt = defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")[:80]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k].add(r.get("Dispatch_Id"))
        for k, m in agg.items():
            n = max(1, len(cnt[k]))
            out.write(f"{k:80s} dispatches {n} " + " ".join(f"{c}={v / n:.4g}" for c, v in sorted(m.items())) + "\n")
out.close()
