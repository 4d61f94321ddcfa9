#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE per k_dense dispatch (two rocprofv3 --pmc
runs of tools/probe_dense_pmc.py), split into its segments, with the gfx950
corrections of MI355X_MICROARCH.md's HBM section (FETCH_SIZE x2 for wide
coalesced 16-B reads; both counters in KiB).

usage: dense_pmc_segments.py FETCH_DIR WRITE_DIR OUT.json [KERNEL]

KERNEL: a substring of the dispatch's kernel name (default "k_dense<false>",
the lung-first stream; "k_dense_persist" for the round-5 runs)
"""
import csv
import glob
import json
import os
import statistics
import sys

# tools/probe_dense_pmc.py's dispatch order: reset() (1), the stagger pre-roll
# (100 x a masked reset + one two-group step: 300), 5 warm steps, the 20-step
# and 64-step windows (two launches per step)
SEGMENTS = [("reset_and_stagger_preroll", 301), ("warm", 10), ("value_window_20_steps", 40),
            ("steady_window_64_steps", 128)]
ENVS, LUNG_VOXELS = 2048, 96160  # per launch; lung voxels of the 64^3 resampled reference mask


def per_dispatch(d, counter, kernel):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                rows.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id")), float(r["Counter_Value"])))
    agg = {}
    for k, v in rows:  # one row per (dispatch, dimension instance) in some versions: sum them
        agg[k] = agg.get(k, 0.0) + v
    return [agg[k] for k in sorted(agg)]


def main(fd, wd, out, kernel="k_dense<false>"):
    f, w = per_dispatch(fd, "FETCH_SIZE", kernel), per_dispatch(wd, "WRITE_SIZE", kernel)
    alg = 4 * LUNG_VOXELS * ENVS
    res = {"kernel": kernel, "envs_per_launch": ENVS, "grid": [64, 64, 64], "lung_voxels": LUNG_VOXELS,
           "dispatches": [len(f), len(w)], "algorithmic_bytes_per_launch": alg,
           "correction": "FETCH_SIZE x2 (gfx950 wide coalesced reads), KiB->B", "segments": {}}
    i = 0
    for name, n in SEGMENTS:
        fs, ws = f[i:i + n], w[i:i + n]
        i += n
        if not fs or not ws:
            continue
        rb, wb = 2 * 1024 * statistics.median(fs), 1024 * statistics.median(ws)
        res["segments"][name] = {"dispatches": len(fs), "read_bytes_median": rb, "write_bytes_median": wb,
                                 "hbm_bytes_median": rb + wb, "traffic_over_algorithmic": (rb + wb) / alg,
                                 "write_bytes_max": 1024 * max(ws)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
