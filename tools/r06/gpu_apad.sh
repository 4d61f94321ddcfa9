#!/bin/bash
# round 6: lung row padding on the final stream: the tree (a16: 64-B sectors)
# against 32-B (a8) and 16-B (a4, no padding past the row's float4) variant
# builds: rollout gates on the tree, the driver's bench alternated, k_dense
# alone + FETCH_SIZE (probe_kdense.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_apad
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_rollout.py tests/test_gpu_configs.py tests/test_gpu_binding.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for t in a16 a8 a4; do
    L=""; [ $t != a16 ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/${t}_$i.json 2> $O/${t}_$i.err || { tail $O/${t}_$i.err; exit 1; }
  done
done
for t in a16 a8 a4; do
  L=""; [ $t != a16 ] && L=$PWD/_var6/librtenv_$t.so
  RT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/pf_$t.log 2>&1 || exit 1
  RT_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ks_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/ks_$t.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, json, statistics, sys
O = sys.argv[1]
for t in ("a16", "a8", "a4"):
    for i in (1, 2):
        d = json.loads([l for l in open(f"{O}/{t}_{i}.json") if l.startswith("{")][-1]); r = d["roofline"]; s = d.get("steady_state", {})
        print(t, i, "value", round(d["value"] / 1e6, 3), "ms", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
              "iso", (r.get("isolated") or {}).get("kernel_ms"), "kd", r.get("kernel_ms"))
    f = []
    for fn in glob.glob(f"{O}/pf_{t}/**/*counter_collection.csv", recursive=True):
        f += [float(r["Counter_Value"]) for r in csv.DictReader(open(fn)) if "k_dense<" in r["Kernel_Name"]]
    for fn in glob.glob(f"{O}/ks_{t}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "k_dense<" in r["Name"]:
                print(t, "k_dense alone avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
    if f:
        print(t, "FETCH x2 median / algorithmic", 2 * 1024 * statistics.median(f) / (4 * 96160 * 4096), "n", len(f))
PY
rm -rf $O/pf_* $O/ks_*
