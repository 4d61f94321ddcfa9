"""Summarise tools/archive/gpu_c3d_pmc.sh: per C3D kernel, median counters over dispatches,
MFMA-busy fraction of SIMD cycles and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs /
kernel time), with the kernel times of the trace pass.

    python tools/c3d_pmc_summary.py gpurun_out/c3dpmc [OUT.json]
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

d = sys.argv[1]
vals = {}
for sub in ("a", "b", "c"):
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "conv" not in k and "dgrad" not in k:
                continue
            k = re.sub(r"\(anonymous namespace\)::", "", k).split("(")[0]
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
times = {}
for f in glob.glob(os.path.join(d, "t", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
        times.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
out = {}
for k, cs in vals.items():
    m = {c: statistics.median(v) for c, v in cs.items()}
    t = statistics.median(times[k]) if k in times else None
    row = dict(m)
    row["kernel_ms"] = t * 1e3 if t else None
    if t and "GRBM_GUI_ACTIVE" in m:
        row["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
    if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"] > 0:
        mf = m["SQ_INSTS_MFMA"]
        row["valu_per_mfma"] = (m["SQ_INSTS_VALU"] - mf) / mf
        row["salu_per_mfma"] = m["SQ_INSTS_SALU"] / mf
        if t and "clock_GHz" in row:
            row["mfma_busy_frac"] = 32 * mf / (1024 * t * row["clock_GHz"] * 1e9)
    if t and "clock_GHz" in row and "SQ_LDS_IDX_ACTIVE" in m:
        # LDS-array cycles over the CU-cycles of the kernel (256 CUs)
        row["lds_active_frac"] = m["SQ_LDS_IDX_ACTIVE"] / (256 * t * row["clock_GHz"] * 1e9)
        if "SQ_LDS_BANK_CONFLICT" in m:
            row["lds_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / max(m["SQ_LDS_IDX_ACTIVE"], 1)
    if t and "clock_GHz" in row and "SQ_INSTS_VALU" in m:
        row["valu_insts_per_cu_cycle"] = m["SQ_INSTS_VALU"] / (256 * t * row["clock_GHz"] * 1e9)
    out[k] = row
    print(f"{k[:60]:60s} ms {row['kernel_ms'] or 0:7.3f} clk {row.get('clock_GHz', 0):5.2f} "
          f"mfma_busy {row.get('mfma_busy_frac', 0):5.3f} valu/mfma {row.get('valu_per_mfma', 0):5.2f} "
          f"salu/mfma {row.get('salu_per_mfma', 0):5.2f} wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / max(m.get('SQ_WAVE_CYCLES', 1), 1):5.2f} "
          f"wait_any {m.get('SQ_WAIT_ANY', 0) / max(m.get('SQ_WAVE_CYCLES', 1), 1):5.2f}")
if len(sys.argv) > 2:
    json.dump({"source": "tools/gpu_r03_s9.sh (or tools/archive/gpu_c3d_pmc.sh) over tools/c3d_pmc_driver.py (batch C3D_PMC_B, 64^3 stage shapes)",
               "kernels": out}, open(sys.argv[2], "w"), indent=1)
