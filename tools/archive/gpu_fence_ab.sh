# pipeline/timing events with vs without the system-scope fence: bench A/B (two passes) + probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fence
rm -f gpurun_out/fence/*
for pass in 1 2; do
  for f in _variants/librtenv_*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update > gpurun_out/fence/${v}_$pass.json 2> gpurun_out/fence/${v}_$pass.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/fence/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "ms step_frac", round(r["step_frac_of_hbm"], 3),
          "frac", round(r["frac"], 3), "timed", round(r["timed_pass_ms_per_step"], 4), "steady", round(d["steady_state"]["env_steps_per_s"] / 1e6, 3),
          "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2))
PY
