#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE) into per-launch HBM
bytes for one kernel, with the gfx950 corrections of MI355X_MICROARCH.md
(HBM section): FETCH_SIZE counts half of a wide coalesced stream's bytes
(x2), both counters are in KiB.

usage: parse_pmc.py FETCH_DIR WRITE_DIR KERNEL OUT.json --grid 64 64 64 --envs 4096
"""
import argparse
import csv
import glob
import json
import os
import statistics


def counter_values(d, kernel, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("kernel")
    ap.add_argument("out")
    ap.add_argument("--grid", type=int, nargs=3, required=True)
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--lung-voxels", type=int, default=0,
                    help="lung-first rows: k_dense reads lung_voxels floats per env (0: the whole volume)")
    a = ap.parse_args()
    f = counter_values(a.fetch_dir, a.kernel, "FETCH_SIZE")
    w = counter_values(a.write_dir, a.kernel, "WRITE_SIZE")
    if not f or not w:
        raise SystemExit(f"no counter rows for {a.kernel}: fetch {len(f)} write {len(w)}")
    fk, wk = statistics.median(f), statistics.median(w)
    V = a.grid[0] * a.grid[1] * a.grid[2]
    out = {
        "kernel": a.kernel, "grid": a.grid, "envs": a.envs, "dispatches": [len(f), len(w)],
        "FETCH_SIZE_KiB_median": fk, "WRITE_SIZE_KiB_median": wk,
        "read_bytes_per_launch": 2 * fk * 1024, "write_bytes_per_launch": wk * 1024,
        "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
        "layout": "lung_first" if a.lung_voxels else "c_order",
        "algorithmic_bytes_per_launch": 4 * (a.lung_voxels or V) * a.envs,
        "correction": "FETCH_SIZE x2 (gfx950 wide coalesced reads), KiB->B",
    }
    out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / out["algorithmic_bytes_per_launch"]
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
