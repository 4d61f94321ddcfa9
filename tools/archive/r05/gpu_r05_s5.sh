#!/bin/bash
# r05 session 5: the tree after conv1's 256-thread default, GAE, the fused
# shuffle + stats and the view-free rollout struct: the GPU suite, smoke, the
# driver's bench command twice, env-group counts 3 / 4, vision f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED|^ERROR" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || { tail -30 $O/bench$i.err; exit 1; }
done
for g in 3 4; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-c3d --no-update --steps 20 --warmup 4 --rollout-groups $g > $O/g$g.json 2> $O/g$g.err || { tail -20 $O/g$g.err; exit 1; }
done
timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_s5"
for i in (1, 2):
    d = json.load(open(f"{O}/bench{i}.json")); r = d["roofline"]; s = d["steady_state"]; c = d["c3d_mfma"]
    print("bench", i, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", round(s["ms_per_step"], 4),
          "vs_value", round(s["vs_value"], 4), "frac", round(r["frac"], 3), "step_frac", round(r["step_frac_of_hbm"], 3),
          "upd f32 us", round(d["ppo_update_ms"] * 1000, 1), "bf16x3", round(d["ppo_update_ms_bf16x3"] * 1000, 1),
          "train", round(d["train_env_steps_per_s"] / 1e6, 2), "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2),
          "incr frac", round(d["other_step_mode"]["roofline"]["frac"], 3), "c3d fwd frac", round(c["forward"]["frac"], 3),
          "train frac", round(c["train_pass"]["frac"], 3), "cpu", d["cpu_baseline"].get("value"))
for g in (3, 4):
    d = json.load(open(f"{O}/g{g}.json")); s = d["steady_state"]
    print("groups", g, round(d["value"] / 1e6, 3), "M steady", round(s["env_steps_per_s"] / 1e6, 3), "M", round(s["ms_per_step"], 4))
d = json.load(open(f"{O}/vision_f32.json"))
print("vision f32: rollout", round(d["value"]), "minibatch ms", round(d["ppo_update_ms"], 2), "iteration", round(d["train_env_steps_per_s"]))
PY
echo ALLDONE
