#!/bin/bash
# round 6: (a) lung rows padded to 16 floats (64 B) instead of 32 (128 B),
# (b) the lane-parallel pose update in k_step_policy (the in-tree library)
# against lp0 (neither): benches alternated, k_dense FETCH_SIZE alone
# (probe_kdense.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r06_a16
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for t in a16 lp0 lane; do
    L=""; [ $t != lane ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/${t}_$i.json 2> $O/${t}_$i.err || exit 1
  done
done
for t in a16 lp0; do
  L=$PWD/_var6/librtenv_$t.so
  RT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/pf_$t.log 2>&1 || exit 1
  RT_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ks_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/ks_$t.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, json, statistics, sys
O = sys.argv[1]
for t in ("a16", "lp0", "lane"):
    for i in (1, 2):
        d = json.load(open(f"{O}/{t}_{i}.json")); r = d["roofline"]; s = d.get("steady_state", {})
        print(t, i, "value", round(d["value"] / 1e6, 3), "ms", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
              "frac", round(r["frac"], 3), "iso", (r.get("isolated") or {}).get("frac"),
              "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 3), "kms", r.get("kernel_ms_all"))
    f = []
    for fn in glob.glob(f"{O}/pf_{t}/**/*counter_collection.csv", recursive=True):
        f += [float(r["Counter_Value"]) for r in csv.DictReader(open(fn)) if "k_dense<" in r["Kernel_Name"]]
    for fn in glob.glob(f"{O}/ks_{t}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "k_dense<" in r["Name"]:
                print(t, "k_dense avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
    alg = 4 * 96160 * 4096
    if f:
        print(t, "FETCH x2 median / algorithmic", 2 * 1024 * statistics.median(f) / alg, "n", len(f))
PY
rm -rf $O/pf_* $O/ks_*
