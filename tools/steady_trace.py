#!/usr/bin/env python3
"""Windows of a rocprofv3 --kernel-trace CSV delimited by one-block
rt_probe_stream marker launches (bench.py steady_state, tools/probe_window.py):
per window the span from its first kernel start to its last kernel end, the
launches and summed durations per kernel, the median k_dense_persist launch
and the time in the span with NO dose stream running.

usage: steady_trace.py KERNEL_TRACE.csv [--labels a,b,c ...]
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)))
    rows.sort()
    return rows


def covered(intervals, lo, hi):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        s, e = max(s, lo), min(e, hi)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--labels", default="")
    a = ap.parse_args()
    rows = load(a.trace)
    marks = [i for i, r in enumerate(rows) if "k_probe_stream" in r[2] and r[3] <= 256]
    labels = a.labels.split(",") if a.labels else []
    out = []
    for w in range(len(marks) - 1):
        ks = rows[marks[w] + 1:marks[w + 1]]
        if not ks:
            continue
        lo, hi = ks[0][0], max(k[1] for k in ks)
        per = defaultdict(lambda: [0, 0.0])
        for s, e, n, _ in ks:
            short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48].strip()
            per[short][0] += 1
            per[short][1] += (e - s) / 1e3
        dense = [(s, e) for s, e, n, _ in ks if "k_dense" in n]
        dd = [(e - s) / 1e3 for s, e in dense]
        rec = {"window": w, "label": labels[w] if w < len(labels) else None, "span_ms": (hi - lo) / 1e6,
               "kernels": {k: {"n": v[0], "sum_us": round(v[1], 1)} for k, v in sorted(per.items())},
               "k_dense_median_us": statistics.median(dd) if dd else None,
               "no_dense_stream_ms": ((hi - lo) - covered(dense, lo, hi)) / 1e6 if dense else None,
               "first_dense_start_us": (dense[0][0] - lo) / 1e3 if dense else None,
               "tail_after_last_dense_us": (hi - max(e for _, e in dense)) / 1e3 if dense else None}
        out.append(rec)
        print(json.dumps(rec))
    return out


if __name__ == "__main__":
    main()
