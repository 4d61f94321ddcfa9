"""Timeline of the dense rollout's kernels from a rocprofv3 kernel trace:
per kernel name and queue, count / mean duration, and one window of steps
listed (start, end relative to the window start) -- to see where the device
hand-off's step time goes (r03 session 24)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
stat = defaultdict(list)
for r in rows:
    stat[(short(r["Kernel_Name"]), r["Queue_Id"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, q), v in sorted(stat.items(), key=lambda x: -sum(x[1])):
    print(f"{k:42s} q{q:>3s} n={len(v):5d} mean {sum(v) / len(v):9.2f} us  total {sum(v) / 1e3:9.2f} ms")
# the last long dense launch and the kernels inside it
dense = [r for r in rows if "k_dense_rollout" in r["Kernel_Name"] or "k_dense_persist" in r["Kernel_Name"]]
if not dense:
    sys.exit()
last = dense[-1]
t0 = int(last["Start_Timestamp"])
if "k_dense_persist" in last["Kernel_Name"]:
    t0 = int(dense[-16]["Start_Timestamp"])
t1 = t0 + int(sys.argv[2] if len(sys.argv) > 2 else 1200) * 1000
print("window from", t0)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 - 50000 and s <= t1:
        print(f"  q{r['Queue_Id']:>3s} {short(r['Kernel_Name']):42s} {(s - t0) / 1e3:9.2f} -> {(e - t0) / 1e3:9.2f}  ({(e - s) / 1e3:8.2f})")
