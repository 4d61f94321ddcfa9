#!/bin/bash
# r05 session 15: kernel statistics of the vision bench (f32), to split the
# 4096-sample minibatch into C3D stages, render and the rest
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s15
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision.json 2> $O/vision.err || { tail -20 $O/vision.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/vision_kernel_stats.csv
rm -rf $O/prof
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05_s15/vision_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot / 1e6, 1))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
echo ALLDONE
