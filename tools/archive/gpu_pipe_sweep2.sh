# pipelined dense rollout knobs after the no-fence events: k_dense_persist blocks per CU x policy block waves (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ps2
rm -f gpurun_out/ps2/*
for pass in 1 2; do
  for bpc in 4 5 6 7; do
    for wpb in 4 8; do
      RT_DENSE_PERSIST=$bpc RT_PIPE_WPB=$wpb timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-update --no-steady --steps 64 > gpurun_out/ps2/b${bpc}_w${wpb}_$pass.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import json, glob, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ps2/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    res[f.split("/")[-1].rsplit("_", 1)[0]].append(d["value"] / 1e6)
for k, v in sorted(res.items()):
    print(k, [round(x, 3) for x in v])
PY
