"""Kernel-to-kernel timeline of a rocprofv3 --kernel-trace database: per
kernel name, mean duration and mean idle gap before it (end of the previous
kernel on the same queue to its start), over a named kernel sequence.

    python tools/rocpd_gaps.py run_results.db k_ppo_grad_mfma k_ppo_reduce k_adam
"""
import sqlite3
import sys
from collections import defaultdict


def main(db, names):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    q = "select name, start, end from kernels order by start"
    rows = list(c.execute(q))
    dur, gap = defaultdict(list), defaultdict(list)
    prev_end = None
    for name, s, e in rows:
        short = next((n for n in names if n in name), None)
        if short:
            dur[short].append((e - s) / 1e3)
            if prev_end is not None and s >= prev_end:
                gap[short].append((s - prev_end) / 1e3)
        prev_end = e
    for n in names:
        d, g = dur[n], gap[n]
        if d:
            d.sort(); g.sort()
            print(f"{n:24s} calls {len(d):5d}  median {d[len(d)//2]:8.2f} us  gap-before median {g[len(g)//2] if g else 0:6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
