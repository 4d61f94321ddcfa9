#!/bin/bash
# round 6 final evidence on the tree, tag $1: the whole GPU suite, smoke, the
# driver's bench command plain (x2) and under rocprofv3 --kernel-trace --stats,
# k_dense FETCH_SIZE / WRITE_SIZE (separate --pmc passes), the bench line
# re-run against the stats of the profiled run, vision f32 at configs[3] and
# configs[4]'s per-GPU share (512 envs x 128^3).  Usage: gpu_final.sh TAG a|b
# (phase a: suite, smoke, profiles; b: the bench lines, which read a's stats
# once copied to profiles/r06/r06_final_kernel_stats.csv)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-final}
PHASE=${2:-a}
O=gpurun_out/r06_$T
mkdir -p $O
if [ "$PHASE" = a ]; then
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/dense_pmc_segments.py $O/pf $O/pw $O/k_dense_pmc.json > /dev/null
rm -rf $O/pf $O/pw
echo PHASE_A_DONE
exit 0
fi
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 tools/probe_dense_pmc.py > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/dense_pmc_segments.py $O/pf $O/pw $O/k_dense_pmc.json > /dev/null
rm -rf $O/pf $O/pw
cp $O/k_dense_pmc.json profiles/r06/r06_final_k_dense_pmc.json  # (this box's copy: the bench lines below read it)
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --rocprof-stats profiles/r06/r06_final_kernel_stats.csv > $O/bench$i.json 2> $O/bench$i.err || { tail -30 $O/bench$i.err; exit 1; }
done
for g in 1 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update --rollout-groups $g > $O/groups$g.json 2> $O/groups$g.err || { tail -30 $O/groups$g.err; exit 1; }
done
timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
timeout -k 10 900 python3 bench.py --vision --grid 128 --num-steps 8 --no-cpu --no-c3d --conv-precision f32 > $O/vision128_f32.json 2> $O/vision128_f32.err || { tail -20 $O/vision128_f32.err; exit 1; }
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for i in (1, 2):
    d = json.loads([l for l in open(f"{O}/bench{i}.json") if l.startswith("{")][-1]); r = d["roofline"]; s = d["steady_state"]
    rp = r.get("rocprof") or {}
    print("bench", i, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", round(s["ms_per_step"], 4),
          "frac", round(r["frac"], 3), "rocprof_ms", rp.get("avg_ms"), "rocprof_frac", rp.get("frac"),
          "traffic", r.get("traffic"), "upd f32 us", round(d["ppo_update_ms"] * 1000, 1),
          "coll", d.get("ppo_update_ms_collective_path"), "train", round(d["train_env_steps_per_s"] / 1e6, 2),
          "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2), "cpu", d["cpu_baseline"].get("value"))
for g in (1, 3):
    d = json.loads([l for l in open(f"{O}/groups{g}.json") if l.startswith("{")][-1]); s = d.get("steady_state", {})
    print("groups", g, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
          "kms", d["roofline"].get("kernel_ms_all"))
for n in ("vision_f32", "vision128_f32"):
    d = json.loads([l for l in open(f"{O}/{n}.json") if l.startswith("{")][-1])
    print(n, "rollout", round(d["value"]), "minibatch ms", round(d["ppo_update_ms"], 2), "iteration", round(d["train_env_steps_per_s"]))
PY
echo ALLDONE
