#!/bin/bash
# r04 session 37 (evidence on the final tree, fourth pass: after the write-through update partials): the whole GPU suite, smoke,
# the driver's bench command plain and under rocprofv3 --kernel-trace --stats,
# k_dense_persist FETCH_SIZE / WRITE_SIZE (separate --pmc passes); c3d.hip is
# unchanged since session 33, whose C3D PMC and vision runs stand
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s37
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/dense_pmc_segments.py $O/pf $O/pw $O/k_dense_persist_pmc.json > /dev/null
rm -rf $O/pf $O/pw
python3 - <<'PY'
import json
O = "gpurun_out/r04_s37"
d = json.load(open(f"{O}/bench.json")); r = d["roofline"]; s = d["steady_state"]
print("bench", round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "timed", round(r["timed_pass_ms_per_step"], 4),
      "steady", round(s["ms_per_step"], 4), "frac", round(r["frac"], 3), "step_frac", round(r["step_frac_of_hbm"], 3),
      "upd f32 us", round(d["ppo_update_ms"] * 1000, 1), "bf16x3", round(d["ppo_update_ms_bf16x3"] * 1000, 1),
      "march", round(r["march"]["frac"], 3), "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2),
      "incr frac", round(d["other_step_mode"]["roofline"]["frac"], 3), "cpu", d["cpu_baseline"].get("value"))
PY
echo ALLDONE
