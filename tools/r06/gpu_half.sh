#!/bin/bash
# round 6: k_dense rows per fetch x waves per SIMD (variant builds in _var6/:
# h10 = 10 rows at 8 waves, h12 = 12 at 7, h16 = 16 at 5; the in-tree library 8 at 8;
# second sweep: h16bN = 16 rows at 5 waves, N blocks per CU in the pipeline, h16w4 = 4 waves, 4 blocks),
# the driver's bench (no cpu / c3d / update) alternated, then k_dense alone (rocprofv3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_half
mkdir -p $O
for i in 1 2; do
  for t in h8 h16b5 h16b4 h16w4; do
    L=""; [ $t != h8 ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/${t}_$i.json 2> $O/${t}_$i.err || { tail $O/${t}_$i.err; exit 1; }
  done
done
for t in h8 h16b5 h16b4 h16w4; do
  L=""; [ $t != h8 ] && L=$PWD/_var6/librtenv_$t.so
  RT_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ks_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/ks_$t.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
for t in ("h8", "h16b5", "h16b4", "h16w4"):
    for i in (1, 2):
        d = json.loads([l for l in open(f"{O}/{t}_{i}.json") if l.startswith("{")][-1]); r = d["roofline"]; s = d.get("steady_state", {})
        print(t, i, "value", round(d["value"] / 1e6, 3), "ms", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
              "iso", (r.get("isolated") or {}).get("kernel_ms"), "kms", r.get("kernel_ms_all"))
    for fn in glob.glob(f"{O}/ks_{t}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "k_dense<" in r["Name"]:
                print(t, "k_dense alone avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
PY
rm -rf $O/ks_*
