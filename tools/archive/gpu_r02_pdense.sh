# persistent dense rollout: bitwise tests, then bench A/B of rollout groups 0 / 2 (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pd
rm -f gpurun_out/pd/*
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pd/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pd/tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for g in 0 2; do
    timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --rollout-groups $g > gpurun_out/pd/bench_g${g}_$pass.json 2> gpurun_out/pd/bench_g${g}_$pass.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/pd/bench_g*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "ms", "frac", round(r["frac"], 3),
          "step_frac", round(r["step_frac_of_hbm"], 3), "steady", round(d["steady_state"]["env_steps_per_s"] / 1e6, 3),
          "train", round(d["train_env_steps_per_s"] / 1e6, 3), "timed_pass", round(r["timed_pass_ms_per_step"], 4))
PY
