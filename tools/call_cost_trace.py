"""Where the per-call cost of the driver's `value` window goes (VERDICT r4
item 4): a rocprofv3 --kernel-trace --hip-runtime-trace of `bench.py` cut at
the first window marker (bench.window_marker: the one-block rt_probe_stream
launched just before the value window's opening synchronise).  The window is
host-timed from the end of that synchronise (t0) to the end of the closing
one (t1); this splits it into
  launch   t0 -> the first k_step_policy starts (host enqueue + dispatch)
  fill     first k_step_policy start -> first k_dense start
  steps    first k_dense start -> last k_dense end (the dose turns + hand-offs)
  drain    last k_dense end -> last kernel end (the last k_finish)
  return   last kernel end -> t1 (the synchronise returning)
and lists the hand-off gaps between consecutive dose turns.

    python tools/call_cost_trace.py <dir with *kernel_trace.csv and *hip_api_trace.csv> [n_steps]
"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
hs = sorted(csv.DictReader(open(ht)), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
mark = next(i for i, r in enumerate(ks) if "k_probe_stream" in r["Kernel_Name"])
win = ks[mark + 1: mark + 1 + 6 * K]  # 2 groups x (k_step_policy, k_dense, k_finish) per step
names = [short(r["Kernel_Name"]) for r in win]
assert names.count("k_dense") == 2 * K, names[:12]
m_end = int(ks[mark]["End_Timestamp"])
syncs = [h for h in hs if "Synchronize" in h["Function"] and int(h["End_Timestamp"]) >= m_end - 10 ** 6]
# the opening synchronise: the first one that ends after the marker kernel ran;
# the closing one: the first that ends after the window's last kernel
last_end = max(int(r["End_Timestamp"]) for r in win)
t0 = int(next(h for h in syncs if int(h["End_Timestamp"]) >= m_end)["End_Timestamp"])
t1 = int(next(h for h in syncs if int(h["End_Timestamp"]) >= last_end)["End_Timestamp"])
first = int(win[0]["Start_Timestamp"])
dense = [r for r in win if short(r["Kernel_Name"]) == "k_dense"]
d0, d1 = int(dense[0]["Start_Timestamp"]), int(dense[-1]["End_Timestamp"])
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(dense, dense[1:])]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in dense]
us = lambda a, b: (b - a) / 1e3
launches = [h for h in hs if int(h["Start_Timestamp"]) >= t0 and int(h["Start_Timestamp"]) <= t1]
enq_end = max((int(h["End_Timestamp"]) for h in launches if "Synchronize" not in h["Function"]), default=t0)
out = {"window_us": us(t0, t1), "per_step_us": us(t0, t1) / K,
       "launch_us": us(t0, first), "fill_us": us(first, d0), "steps_us": us(d0, d1), "drain_us": us(d1, last_end),
       "return_us": us(last_end, t1), "host_enqueue_us": us(t0, enq_end), "hip_calls_in_window": len(launches),
       "dense_turn_us_median": statistics.median(durs), "handoff_gap_us_median": statistics.median(gaps),
       "handoff_gap_us_max": max(gaps), "steps_per_step_us": us(d0, d1) / K}
for k, v in out.items():
    print(f"{k:24s} {v:10.2f}" if isinstance(v, float) else f"{k:24s} {v}")
# the host side of the window's head and tail: every HIP API call between the
# opening synchronise and the first kernel, and after the last launch
print("-- HIP calls from t0 (us: start, end, function); first kernel at", round(us(t0, first), 2))
for h in hs:
    s0, e0 = int(h["Start_Timestamp"]), int(h["End_Timestamp"])
    if t0 - 50_000 <= s0 <= first + 20_000:
        print(f"  {us(t0, s0):9.2f} {us(t0, e0):9.2f}  {h['Function']}")
print("-- HIP calls around the last kernel end (", round(us(t0, last_end), 2), ") and t1 (", round(us(t0, t1), 2), ")")
for h in hs:
    s0, e0 = int(h["Start_Timestamp"]), int(h["End_Timestamp"])
    if last_end - 60_000 <= e0 <= t1 + 1_000:
        print(f"  {us(t0, s0):9.2f} {us(t0, e0):9.2f}  {h['Function']}")
