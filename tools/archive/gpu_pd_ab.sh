# persistent dense rollout variants (_variants/librtenv_pd*.so) vs the pipelined default, bench A/B (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pdab
rm -f gpurun_out/pdab/*
for pass in 1 2; do
  for f in _variants/librtenv_pd*.so; do
    v=$(basename $f .so)
    RT_LIB_PATH=$f timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update --no-steady --rollout-groups 0 > gpurun_out/pdab/${v}_$pass.json 2> gpurun_out/pdab/${v}_$pass.err || exit 1
  done
  timeout -k 10 300 python -u bench.py --no-cpu --no-c3d --no-update --no-steady --rollout-groups 2 > gpurun_out/pdab/g2_$pass.json 2> gpurun_out/pdab/g2_$pass.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/pdab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 3), "M", round(d["ms_per_step"], 4), "ms step_frac", round(r["step_frac_of_hbm"], 3))
PY
