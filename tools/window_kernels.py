"""Cut a rocprofv3 kernel trace (CSV) at the one-block rt_probe_stream marker
launches (tools/probe_first_window.py, bench.py's steady-state windows) and
summarise each window: span from its first to its last kernel, kernels per
name (count, mean and total duration), and the time the dose stream
(k_dense_persist) was idle between its launches.

    python tools/window_kernels.py kernel_trace.csv [--max-windows N]"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:34]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_probe_stream" in r["Kernel_Name"]
             and int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0) <= 256]
    out = []
    for w, (a, b) in enumerate(zip(marks, marks[1:])):
        ks = rows[a + 1:b]
        if not ks:
            continue
        t0 = int(ks[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in ks)
        per = defaultdict(list)
        for r in ks:
            per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        dense = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "k_dense" in r["Kernel_Name"]]
        idle = sum(max(0, s1 - e0) for (_, e0), (s1, _) in zip(dense, dense[1:])) / 1e3
        print(f"window {w}: span {(t1 - t0) / 1e3:9.1f} us, dense idle {idle:8.1f} us, kernels {len(ks)}")
        for k, v in sorted(per.items(), key=lambda x: -sum(x[1])):
            print(f"    {k:34s} n={len(v):4d} mean {sum(v) / len(v):8.2f} us total {sum(v):9.1f} us")
        out.append((t1 - t0) / 1e3)
    return out


if __name__ == "__main__":
    main()
