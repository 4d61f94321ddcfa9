#!/bin/bash
# r05 session 8: groups-2 data gradient in 6-wave blocks (3 waves per SIMD)
# vs the 4-wave build (variant dg256): C3D gates, stage times, vision f32;
# then the full GPU suite, smoke and the driver's bench command on the tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1 || { tail -40 $O/pytest_c3d.log; exit 1; }
tail -1 $O/pytest_c3d.log
for v in base dg256; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v = dg256 ] && L=_variants/librtenv_dg256.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_$v.txt 2> $O/stages_$v.err || { tail -20 $O/stages_$v.err; exit 1; }
  grep -v "^{" $O/stages_$v.txt | head -12
done
for v in base dg256; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v = dg256 ] && L=_variants/librtenv_dg256.so
  RT_LIB_PATH=$L timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_$v.json 2> $O/vision_$v.err || { tail -20 $O/vision_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/vision_$v.json'))
print('$v vision f32: rollout', round(d['value']), 'minibatch ms', round(d['ppo_update_ms'],2), 'iteration', round(d['train_env_steps_per_s']))"
done
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit 1
grep -E "^FAILED|^ERROR" $O/pytest_gpu.log || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05_s8/bench.json")); r = d["roofline"]; s = d["steady_state"]; c = d["c3d_mfma"]
print("bench", round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "steady", round(s["ms_per_step"], 4),
      "vs_value", round(s["vs_value"], 4), "frac", round(r["frac"], 3), "step_frac", round(r["step_frac_of_hbm"], 3),
      "upd f32 us", round(d["ppo_update_ms"] * 1000, 1), "train", round(d["train_env_steps_per_s"] / 1e6, 2),
      "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2), "incr frac", round(d["other_step_mode"]["roofline"]["frac"], 3),
      "cpu", d["cpu_baseline"].get("value"))
PY
echo ALLDONE
