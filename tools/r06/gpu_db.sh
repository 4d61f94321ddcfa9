#!/bin/bash
# round 6: k_dense with two chain groups in flight per wave (double-buffered
# fetch, branch-free out-of-range row masking; db3 = 3 waves per SIMD, 3
# blocks per CU in the pipeline), the branch-free masking alone (oob, 16 rows
# at 5 waves) and the in-tree library (cur): the rollout gates on db3, the
# driver's bench alternated, then k_dense alone (rocprofv3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_db
mkdir -p $O
RT_LIB_PATH=$PWD/_var6/librtenv_db3.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_rollout.py tests/test_gpu_configs.py > $O/pytest_db3.log 2>&1 || { tail -20 $O/pytest_db3.log; exit 1; }
tail -1 $O/pytest_db3.log
for i in 1 2; do
  for t in cur oob db3; do
    L=""; [ $t != cur ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/${t}_$i.json 2> $O/${t}_$i.err || { tail $O/${t}_$i.err; exit 1; }
  done
done
for t in cur oob db3; do
  L=""; [ $t != cur ] && L=$PWD/_var6/librtenv_$t.so
  RT_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/ks_$t -o kd --output-format csv -- python3 tools/r06/probe_kdense.py > $O/ks_$t.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
for t in ("cur", "oob", "db3"):
    for i in (1, 2):
        d = json.loads([l for l in open(f"{O}/{t}_{i}.json") if l.startswith("{")][-1]); r = d["roofline"]; s = d.get("steady_state", {})
        print(t, i, "value", round(d["value"] / 1e6, 3), "ms", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
              "iso", (r.get("isolated") or {}).get("kernel_ms"), "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2),
              "kms", r.get("kernel_ms_all"))
    for fn in glob.glob(f"{O}/ks_{t}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "k_dense<" in r["Name"]:
                print(t, "k_dense alone avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
PY
rm -rf $O/ks_*
