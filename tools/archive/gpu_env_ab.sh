# HIP runtime environment knobs: bench A/B (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/envab
rm -f gpurun_out/envab/*
for pass in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update --no-steady > gpurun_out/envab/base_$pass.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update --no-steady > gpurun_out/envab/devkernarg1_$pass.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update --no-steady > gpurun_out/envab/devkernarg0_$pass.json 2>/dev/null || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/envab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "ms step_frac", round(r["step_frac_of_hbm"], 3),
          "incr", round(d["other_step_mode"]["env_steps_per_s"] / 1e6, 2))
PY
